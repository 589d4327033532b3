#!/bin/bash
# Config-2 sweep: VALU plan block count (RFX_VALU_BLOCKS) x one-launch / three-launch search, after
# the VALU parity tests.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/cfg2"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_filters.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 300 --no-cpu-baseline --oracle-stride 0"
for B in ${BLOCKS:-256 384 512 768 1024 old}; do
  for F in "" "--unfused"; do
    if [ "$B" = old ]; then E="RFX_VALU_RPW=64"; else E="RFX_VALU_BLOCKS=$B"; fi
    env $E timeout -k 10 120 python -u bench.py $C2 $F > "$O/b_${B}${F}.log" 2>&1 || { tail -20 "$O/b_${B}${F}.log"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3] or 'fused', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/b_${B}${F}.log" "$B" "$F"
  done
done
echo "== done $(date +%T)"
