#!/bin/bash
# round 3: kernel 11 at config 2: copies 1 vs 8 (cache-resident vs HBM), ablations, and 200k / 400k rows
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03r; mkdir -p $O
C2="--dim 768 --dtype f32 --nq 1 --k 10 --steps 2000 --warmup 50 --event-stride 16 --no-cpu-baseline --oracle-stride 0"
for cfg in "--rows 100000 --copies 1" "--rows 100000 --copies 8" "--rows 400000" "--rows 1600000"; do
  for m in 0 8 10; do
    RFX_K11_ABLATE=$m timeout -k 10 200 python -u bench.py $C2 $cfg > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "$cfg ablate $m: $(grep -o '"ms_per_step": [0-9.]*' $O/b.log) $(grep -o '"kernel_ms": [0-9.]*' $O/b.log)"
  done
  timeout -k 10 200 python -u bench.py $C2 $cfg --scan exact > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg exact: $(grep -o '"ms_per_step": [0-9.]*' $O/b.log) $(grep -o '"kernel_ms": [0-9.]*' $O/b.log)"
done
