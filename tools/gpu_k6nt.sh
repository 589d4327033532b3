#!/bin/bash
# Kernel 6 (4-slot ring): non-temporal corpus DMA (production) against the default policy (debug
# MODE 16) at config 3, bursts interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k6nt}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u tools/k5_variants.py --rows 10000000 --modes 3,20000016 --rounds 8 --burst 30 --no-stream-ref > "$O/cfg3.json" 2> "$O/cfg3.err" || { tail -20 "$O/cfg3.err"; exit 1; }
cat "$O/cfg3.json"
