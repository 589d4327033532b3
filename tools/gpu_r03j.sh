#!/bin/bash
# round 3 (re-entry): two-pass parity tests, config-3 bench two-pass and exact, rocprofv3 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_screen.py > $O/pytest_screen.log 2>&1 || { tail -30 $O/pytest_screen.log; exit 1; }
tail -3 $O/pytest_screen.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_screen.log 2>&1 || { tail -20 $O/bench_screen.log; exit 1; }
tail -c 3000 $O/bench_screen.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --scan exact --no-cpu-baseline > $O/bench_exact.log 2>&1 || { tail -20 $O/bench_exact.log; exit 1; }
tail -c 1500 $O/bench_exact.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --oracle-stride 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -12 {} \;
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 700 --timeout-method thread tests/test_gpu_ivf_cfg5.py > $O/pytest_cfg5.log 2>&1 || { tail -30 $O/pytest_cfg5.log; exit 1; }
tail -6 $O/pytest_cfg5.log
