#!/bin/bash
# Kernel 7 (d = 1024, config 4 shard) on one GPU: its parity tests, the 12.5M×1024 f16 shard bench
# (oracle-checked) with and without the non-temporal DMA hint, kernel stats and FETCH_SIZE passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k7}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filters.py -m gpu -k "k7 or 1024 or every_kernel or mfma_batched" -x -q --timeout 300 --timeout-method thread > "$O/pytest_k7.log" 2>&1 || { tail -40 "$O/pytest_k7.log"; exit 1; }
tail -2 "$O/pytest_k7.log"
fi
C4="--rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline"
step bench
timeout -k 10 300 python -u bench.py $C4 --steps 20 --warmup 3 --oracle-stride 16 > "$O/bench_cfg4.log" 2>&1 || { tail -20 "$O/bench_cfg4.log"; exit 1; }
tail -1 "$O/bench_cfg4.log" | cut -c1-900
step bench_mode16
RFX_K7_MODE=16 timeout -k 10 300 python -u bench.py $C4 --steps 20 --warmup 3 --oracle-stride 64 > "$O/bench_cfg4_m16.log" 2>&1 || { tail -20 "$O/bench_cfg4_m16.log"; exit 1; }
tail -1 "$O/bench_cfg4_m16.log" | cut -c1-900
cd /tmp && export TMPDIR=/tmp
step kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt4" -o kt4 -- python "$R/bench.py" $C4 --steps 20 --warmup 3 --oracle-stride 0 > "$O/bench_kt4.log" 2>&1 || { tail -20 "$O/bench_kt4.log"; exit 1; }
step pmc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf4" -o pmcf4 -- python "$R/bench.py" $C4 --steps 5 --warmup 1 --oracle-stride 0 > "$O/bench_pmcf4.log" 2>&1 || { tail -20 "$O/bench_pmcf4.log"; exit 1; }
export RFX_K7_MODE=16
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf4m16" -o pmcf4m16 -- python "$R/bench.py" $C4 --steps 5 --warmup 1 --oracle-stride 0 > "$O/bench_pmcf4m16.log" 2>&1 || { tail -20 "$O/bench_pmcf4m16.log"; exit 1; }
step done
