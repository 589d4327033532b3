#!/bin/bash
# Kernel 9 (batched f32 scan) on one GPU: parity tests, then the bench at 10M×768 f32, nq 256, k 10
# (oracle-checked) with kernel stats.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-k9}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filters.py tests/test_gpu_fused.py tests/test_gpu_boundary.py tests/test_gpu_merge.py -m gpu -k "f32 or every_kernel or ranges or fused or boundary or merge" -x -q --timeout 300 --timeout-method thread > "$O/pytest_k9.log" 2>&1 || { tail -40 "$O/pytest_k9.log"; exit 1; }
tail -2 "$O/pytest_k9.log"
fi
step bench
timeout -k 10 400 python -u bench.py --rows 10000000 --dim 768 --dtype f32 --no-cpu-baseline --steps 5 --warmup 1 --oracle-stride 16 > "$O/bench_f32_10m.log" 2>&1 || { tail -20 "$O/bench_f32_10m.log"; exit 1; }
tail -1 "$O/bench_f32_10m.log" | cut -c1-300
timeout -k 10 300 python -u bench.py --rows 100000 --dim 768 --dtype f32 --nq 64 --no-cpu-baseline --steps 200 --warmup 20 --oracle-stride 8 > "$O/bench_f32_100k_nq64.log" 2>&1 || { tail -20 "$O/bench_f32_100k_nq64.log"; exit 1; }
tail -1 "$O/bench_f32_100k_nq64.log" | cut -c1-300
cd /tmp && export TMPDIR=/tmp
step kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python "$R/bench.py" --rows 10000000 --dim 768 --dtype f32 --no-cpu-baseline --steps 5 --warmup 1 --oracle-stride 0 > "$O/bench_kt.log" 2>&1 || { tail -20 "$O/bench_kt.log"; exit 1; }
step done
