#!/bin/bash
# Round 6: kernel-10 A/B in the debug library (interleaved bursts, answers checked equal to production):
# production 1010485760 against the variants given (default: one wave DMAs the tile records, 1044040192),
# at 10M rows and at the 8-GPU shard (1.25M rows).
set -o pipefail
O=${1:-gpurun_out/r06k}; V=${2:-1010485760,1044040192}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/k10_variants.py --variants $V --rounds 6 --burst 30 --validate > "$O/ab_10m.json" 2> "$O/ab_10m.err" || { echo "10m rc=$?"; tail -5 "$O/ab_10m.err"; exit 1; }
tail -25 "$O/ab_10m.json"
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants $V --rounds 6 --burst 100 --validate > "$O/ab_shard.json" 2> "$O/ab_shard.err" || { echo "shard rc=$?"; tail -5 "$O/ab_shard.err"; exit 1; }
tail -25 "$O/ab_shard.json"
