#!/bin/bash
# round 4: kernel 10's slow-path entries and trips by tile index (debug MODE 8192), shard and 10M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z7; mkdir -p $O
timeout -k 10 240 python -u tools/k10_trips.py --rows 1250000 > $O/k10_trips_shard.json 2>&1 || { tail -20 $O/k10_trips_shard.json; exit 1; }
grep -v amdgpu $O/k10_trips_shard.json | tr -d ' \n'; echo
timeout -k 10 300 python -u tools/k10_trips.py --rows 10000000 --reps 3 > $O/k10_trips_10m.json 2>&1 || { tail -20 $O/k10_trips_10m.json; exit 1; }
grep -v amdgpu $O/k10_trips_10m.json | tr -d ' \n'; echo
