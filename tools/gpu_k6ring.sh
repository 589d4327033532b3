#!/bin/bash
# kernel 6: is the stream latency-bound?  KL 4 lists with a 6- vs 7-slot ring (k = 4), and the
# k = 10 production kernel, back-to-back bursts.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/k6ring"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u tools/k5_variants.py --k 4 --modes 3,20000070,20000071 > "$O/k4.json" 2> "$O/k4.err" || { tail -30 "$O/k4.err"; exit 1; }
cat "$O/k4.json"
timeout -k 10 300 python -u tools/k5_variants.py --modes 3,132072,20000000 > "$O/k10.json" 2> "$O/k10.err" || { tail -30 "$O/k10.err"; exit 1; }
cat "$O/k10.json"
