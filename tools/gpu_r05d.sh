#!/bin/bash
# round 5: kernel 10 with one wait + barrier per tile (debug TB) on round 4's fold; the sharded search's
# per-shard Python path against the one-call C path (a corrupted record seen in r05c)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python -u tools/debug_sharded_paths.py > $O/debug_sharded_paths.log 2>&1 || { tail -30 $O/debug_sharded_paths.log; }
grep -v amdgpu $O/debug_sharded_paths.log | head -40
V=80000000,122097152,102097152,122621440,122097664,122097153
timeout -k 10 500 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_shard.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 500 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_10m.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 300 python -u tools/k10_trips.py --variant 122105344 > $O/k10_trips_tb.json 2>&1 || { tail -20 $O/k10_trips_tb.json; exit 1; }
timeout -k 10 300 python -u tools/k10_trips.py --variant 80008192 > $O/k10_trips_prod.json 2>&1 || { tail -20 $O/k10_trips_prod.json; exit 1; }
grep -h "total" $O/k10_trips_*.json
