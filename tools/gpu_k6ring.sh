#!/bin/bash
# Kernel 6 ring-depth sensitivity at config 3: the production library (6-slot ring) against side
# builds with 5- and 4-slot rings (librfx_k6r{5,4}.so, -DRFX_K6_RING=N), alternating.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k6ring}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
C3="--no-cpu-baseline --steps 40 --warmup 5 --oracle-stride 0"
for i in 1 2; do
  for v in prod k6r5 k6r4; do
    L="$R/rag-foundation_amd/rfx/librfx_$v.so"; [ "$v" = prod ] && L="$R/rag-foundation_amd/rfx/librfx.so"
    RFX_LIB="$L" timeout -k 10 200 python -u bench.py $C3 > "$O/${v}_$i.log" 2>&1 || { tail -20 "$O/${v}_$i.log"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/${v}_$i.log" ${v}_$i
  done
done
for v in k6r5 k6r4; do  # the shard shape of the 8-GPU run
  L="$R/rag-foundation_amd/rfx/librfx_$v.so"
  RFX_LIB="$L" timeout -k 10 200 python -u bench.py --rows 1250000 $C3 > "$O/${v}_shard.log" 2>&1 || { tail -20 "$O/${v}_shard.log"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/${v}_shard.log" ${v}_shard
done
timeout -k 10 200 python -u bench.py --rows 1250000 $C3 > "$O/prod_shard.log" 2>&1 || { tail -20 "$O/prod_shard.log"; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/prod_shard.log" prod_shard
