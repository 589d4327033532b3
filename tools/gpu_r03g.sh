#!/bin/bash
# round 3: kernel 10 v2 (integer fast path, no per-tile loads, PF 2): parity tests, variants, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_screen.py > $O/pytest_screen.log 2>&1 || { tail -30 $O/pytest_screen.log; exit 1; }
tail -3 $O/pytest_screen.log
timeout -k 10 400 python -u tools/k10_variants.py --variants 800,804,802,400,404,1000,801,809,9 > $O/variants.json 2> $O/variants.err || { tail -5 $O/variants.err; exit 1; }
cat $O/variants.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -c 2500 $O/bench.log
