#!/bin/bash
# Kernel 8 ring-depth sensitivity: the production library (5-slot ring) against a side build with
# a 4-slot ring (librfx_ring4.so, -DRFX_K8_RING=4), alternating, at the config-4 shard.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k8ring}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
C4="--rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 30 --warmup 5 --oracle-stride 0"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $C4 > "$O/prod_$i.log" 2>&1 || { tail -20 "$O/prod_$i.log"; exit 1; }
  RFX_LIB="$R/rag-foundation_amd/rfx/librfx_ring4.so" timeout -k 10 200 python -u bench.py $C4 > "$O/ring4_$i.log" 2>&1 || { tail -20 "$O/ring4_$i.log"; exit 1; }
  for f in prod_$i ring4_$i; do
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/$f.log" $f
  done
done
