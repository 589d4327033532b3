#!/bin/bash
# round 3: config 3 bench, two-pass (default) vs exact, + rocprofv3 kernel stats of the default run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r03b_bench_screen.log 2>&1 || { tail -20 gpurun_out/r03b_bench_screen.log; exit 1; }
tail -c 3000 gpurun_out/r03b_bench_screen.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --scan exact --no-cpu-baseline > gpurun_out/r03b_bench_exact.log 2>&1 || { tail -20 gpurun_out/r03b_bench_exact.log; exit 1; }
tail -c 1500 gpurun_out/r03b_bench_exact.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b_prof -o run -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --oracle-stride 0 > gpurun_out/r03b_prof.log 2>&1 || { tail -20 gpurun_out/r03b_prof.log; exit 1; }
find gpurun_out/r03b_prof -name "*kernel_stats.csv" | head -3
