#!/bin/bash
# round 3: kernel 10's slow path as a per-lane pop loop over a pass mask (8000) against the serial
# LDS insert (9024) and the slow path never taken (8512); two-pass GPU tests; config-3 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --variants 8000,9024,8512,8000,9024 --rounds 4 > $O/k10_variants.txt 2>&1 || { tail -20 $O/k10_variants.txt; exit 1; }
cat $O/k10_variants.txt | tail -15
timeout -k 10 600 python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -c 1500 $O/bench.log
