#!/bin/bash
# d = 1024 kernels on one GPU: parity tests of the production kernel, the 12.5M×1024 f16 config-4
# shard bench (oracle-checked) for kernel 8 (k-split pairs) and kernel 7, kernel stats and FETCH_SIZE.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k8}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filters.py -m gpu -k "d1024 or 1024 or every_kernel or mfma_batched" -x -q --timeout 300 --timeout-method thread > "$O/pytest_d1024.log" 2>&1 || { tail -40 "$O/pytest_d1024.log"; exit 1; }
tail -2 "$O/pytest_d1024.log"
fi
C4="--rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline"
step bench_k8
timeout -k 10 300 python -u bench.py $C4 --steps 20 --warmup 3 --oracle-stride 16 > "$O/bench_cfg4_k8.log" 2>&1 || { tail -20 "$O/bench_cfg4_k8.log"; exit 1; }
tail -1 "$O/bench_cfg4_k8.log" | cut -c1-300
step bench_k7
RFX_D1024_KERNEL=7 timeout -k 10 300 python -u bench.py $C4 --steps 20 --warmup 3 --oracle-stride 64 > "$O/bench_cfg4_k7.log" 2>&1 || { tail -20 "$O/bench_cfg4_k7.log"; exit 1; }
tail -1 "$O/bench_cfg4_k7.log" | cut -c1-300
step cfg2_events
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 300 --no-cpu-baseline --oracle-stride 0"
for E in 1 16; do
  timeout -k 10 300 python -u bench.py $C2 --event-stride $E > "$O/bench_cfg2_ev$E.log" 2>&1 || { tail -20 "$O/bench_cfg2_ev$E.log"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ev', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/bench_cfg2_ev$E.log" $E
done
cd /tmp && export TMPDIR=/tmp
step kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt4" -o kt4 -- python "$R/bench.py" $C4 --steps 20 --warmup 3 --oracle-stride 0 > "$O/bench_kt4.log" 2>&1 || { tail -20 "$O/bench_kt4.log"; exit 1; }
step pmc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf4" -o pmcf4 -- python "$R/bench.py" $C4 --steps 5 --warmup 1 --oracle-stride 0 > "$O/bench_pmcf4.log" 2>&1 || { tail -20 "$O/bench_pmcf4.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmcw4" -o pmcw4 -- python "$R/bench.py" $C4 --steps 5 --warmup 1 --oracle-stride 0 > "$O/bench_pmcw4.log" 2>&1 || { tail -20 "$O/bench_pmcw4.log"; exit 1; }
step done
