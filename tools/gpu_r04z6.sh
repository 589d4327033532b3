#!/bin/bash
# round 4: the 2-rank bench rehearsal as a pytest (rank-0 oracle check of the gathered answer)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z6; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_bench_rehearsal.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -4 $O/pytest.log
