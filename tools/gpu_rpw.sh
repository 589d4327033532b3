#!/bin/bash
# Config-2 rows-per-wave sweep of scan_valu_kernel (RFX_VALU_RPW), then parity tests at rpw 32.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
export PYTHONDONTWRITEBYTECODE=1
C2="--rows 100000 --dim 768 --nq 1 --dtype f32 --no-cpu-baseline --steps 3000 --warmup 100"
: > "$O/rpw_sweep.log"
for r in 64 16 32 48 128 64; do
  RFX_VALU_RPW=$r timeout -k 10 120 python bench.py $C2 > "$O/bench_rpw.log" 2>&1 || { echo "rpw $r rc=$?"; tail -20 "$O/bench_rpw.log"; exit 1; }
  echo "rpw $r $(tail -1 "$O/bench_rpw.log" | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"])')" >> "$O/rpw_sweep.log"
done
cat "$O/rpw_sweep.log"
RFX_VALU_RPW=32 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filters.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_rpw.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$O/pytest_rpw.log"; exit 1; }
tail -1 "$O/pytest_rpw.log"
