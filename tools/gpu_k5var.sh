#!/bin/bash
# headline-kernel ablations (debug library), back-to-back bursts; then the production bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/k5var"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u tools/k5_variants.py ${ARGS} > "$O/variants.json" 2> "$O/variants.err" || { tail -30 "$O/variants.err"; exit 1; }
cat "$O/variants.json"
