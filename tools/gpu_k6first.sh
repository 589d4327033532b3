#!/bin/bash
# Kernel 6 first-tile ablations (debug library): timing and exact-row checks at the 8-GPU shard
# (1.25M rows) and at config 3 (10M rows).  MODE 64: no slot publication at tile 0; 256: tile 0
# folded by rank; 320: both.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k6first}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
M=3,20000064,20000256,20000320
timeout -k 10 300 python -u tools/k5_variants.py --rows 1250000 --modes $M --rounds 6 --burst 100 --no-stream-ref > "$O/shard.json" 2> "$O/shard.err" || { tail -20 "$O/shard.err"; exit 1; }
cat "$O/shard.json"
timeout -k 10 400 python -u tools/k5_variants.py --rows 10000000 --modes $M --rounds 4 --burst 20 --no-stream-ref > "$O/cfg3.json" 2> "$O/cfg3.err" || { tail -20 "$O/cfg3.err"; exit 1; }
cat "$O/cfg3.json"
