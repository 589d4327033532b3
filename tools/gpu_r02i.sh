#!/bin/bash
# Round-2 GPU session I: smoke, the -m gpu suite, the default bench (config 3), config 2 with kernel
# stats, the config-4 shard (12.5M rows, oracle-checked) and config 4 whole on one GPU (100M×1024
# f16 = 204.8 GB, the 1-GPU reference point of SURVEY §8d; no oracle pass at that size).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-r02i}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=8 -q --timeout 420 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
fi
step bench
timeout -k 10 400 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
step cfg2
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 300 --event-stride 16"
timeout -k 10 300 python -u bench.py $C2 > "$O/bench_cfg2.log" 2>&1 || { tail -20 "$O/bench_cfg2.log"; exit 1; }
tail -1 "$O/bench_cfg2.log" | cut -c1-200
step cfg4_shard
timeout -k 10 300 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 20 --warmup 3 --oracle-stride 16 > "$O/bench_cfg4_shard.log" 2>&1 || { tail -20 "$O/bench_cfg4_shard.log"; exit 1; }
tail -1 "$O/bench_cfg4_shard.log" | cut -c1-200
step cfg4_whole
timeout -k 10 400 python -u bench.py --rows 100000000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 5 --warmup 1 --oracle-stride 0 > "$O/bench_cfg4_whole.log" 2>&1 || { tail -20 "$O/bench_cfg4_whole.log"; exit 1; }
tail -1 "$O/bench_cfg4_whole.log" | cut -c1-200
cd /tmp && export TMPDIR=/tmp
step kt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt2 -- python "$R/bench.py" $C2 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt2.log" 2>&1 || { tail -20 "$O/bench_kt2.log"; exit 1; }
step done
