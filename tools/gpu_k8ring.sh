#!/bin/bash
# Kernel 8 ring-depth sensitivity: the production library (5-slot ring) against side builds with
# 4- and 3-slot rings (librfx_ring{4,3}.so, -DRFX_K8_RING=N), alternating, at the config-4 shard.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k8ring}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
C4="--rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 30 --warmup 5 --oracle-stride 0"
for i in 1 2; do
  for v in prod ring4 ring3; do
    L="$R/rag-foundation_amd/rfx/librfx_$v.so"; [ "$v" = prod ] && L="$R/rag-foundation_amd/rfx/librfx.so"
    RFX_LIB="$L" timeout -k 10 200 python -u bench.py $C4 > "$O/${v}_$i.log" 2>&1 || { tail -20 "$O/${v}_$i.log"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/${v}_$i.log" ${v}_$i
  done
done
