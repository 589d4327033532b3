#!/bin/bash
# kernel-6 bring-up: parity (GPU suite subset incl. full size), then ablation timings vs kernel 5.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/k6"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_filters.py tests/test_gpu_fullsize.py} -m gpu --maxfail=5 -q --timeout 420 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 400 python -u tools/k5_variants.py > "$O/variants.json" 2> "$O/variants.err" || { tail -30 "$O/variants.err"; exit 1; }
cat "$O/variants.json"
