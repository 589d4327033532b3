#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 400 python -u tools/k10_variants.py --variants 832,800,801,809,400,1000,9 --rounds 3 > $O/variants.json 2> $O/variants.err || { tail -5 $O/variants.err; exit 1; }
cat $O/variants.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_screen.py > $O/pytest_screen.log 2>&1 || { tail -30 $O/pytest_screen.log; exit 1; }
tail -2 $O/pytest_screen.log
