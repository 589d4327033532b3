#!/bin/bash
# Round 6: smoke and the whole -m gpu suite on one box (the full-size oracle checks included).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${1:-gpurun_out/r06g}; mkdir -p $O
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -60 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
