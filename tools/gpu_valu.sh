#!/bin/bash
# VALU scan changes on one GPU: VALU / one-launch / filter / merge parity tests, then the config-2
# bench (rotating copies, events on every 16th step) with kernel stats.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-valu}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_filters.py tests/test_gpu_merge.py -m gpu -k "valu or cfg2 or fused or every_kernel or f32 or tomb or merge" -x -q --timeout 300 --timeout-method thread > "$O/pytest_valu.log" 2>&1 || { tail -40 "$O/pytest_valu.log"; exit 1; }
tail -2 "$O/pytest_valu.log"
fi
step cfg2
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 300 --event-stride 16"
timeout -k 10 300 python -u bench.py $C2 > "$O/bench_cfg2.log" 2>&1 || { tail -20 "$O/bench_cfg2.log"; exit 1; }
tail -1 "$O/bench_cfg2.log" | cut -c1-200
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['oracle_check']['ok'])" "$O/bench_cfg2.log"
cd /tmp && export TMPDIR=/tmp
step kt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt2 -- python "$R/bench.py" $C2 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt2.log" 2>&1 || { tail -20 "$O/bench_kt2.log"; exit 1; }
step done
