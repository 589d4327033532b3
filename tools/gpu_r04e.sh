#!/bin/bash
# round 4: the full GPU suite on the new select / merge / re-score code, then the tie debug
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 1050 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u tools/debug_sharded_ties.py > $O/ties.log 2>&1 || { tail -30 $O/ties.log; exit 1; }
tail -3 $O/ties.log
