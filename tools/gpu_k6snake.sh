#!/bin/bash
# Kernel 6 MFMA issue order (debug MODE 512: snake order) against production at config 3, bursts.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k6snake}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u tools/k5_variants.py --rows 10000000 --modes 3,20000512 --rounds 8 --burst 30 --no-stream-ref > "$O/cfg3.json" 2> "$O/cfg3.err" || { tail -20 "$O/cfg3.err"; exit 1; }
cat "$O/cfg3.json"
