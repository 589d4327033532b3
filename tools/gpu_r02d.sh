#!/bin/bash
# Round-2 GPU session D: the -m gpu suite, config-2 bench (one launch) with kernel stats and FETCH,
# and the per-rank shard shapes of the N = 2, 4, 8 scaling runs (config 3 split over N GPUs) with
# kernel stats of the 8-GPU shard.  Every GPU step has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02d"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=8 -q --timeout 420 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
fi
step cfg2
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 300"
timeout -k 10 300 python -u bench.py $C2 > "$O/bench_cfg2.log" 2>&1 || { tail -20 "$O/bench_cfg2.log"; exit 1; }
tail -1 "$O/bench_cfg2.log" | cut -c1-200
step shards
for N in 1250000 2500000 5000000; do
  timeout -k 10 300 python -u bench.py --rows $N --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 16 > "$O/bench_rows$N.log" 2>&1 || { tail -20 "$O/bench_rows$N.log"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['oracle_check']['ok'])" "$O/bench_rows$N.log" $N
done
cd /tmp && export TMPDIR=/tmp
step kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt2 -- python "$R/bench.py" $C2 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt2.log" 2>&1 || { tail -20 "$O/bench_kt2.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf2" -o pmcf2 -- python "$R/bench.py" --rows 100000 --dim 768 --dtype f32 --nq 1 --steps 50 --warmup 10 --no-cpu-baseline --oracle-stride 0 > "$O/bench_pmcf2.log" 2>&1 || { tail -20 "$O/bench_pmcf2.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt8" -o kt8 -- python "$R/bench.py" --rows 1250000 --steps 100 --warmup 10 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt8.log" 2>&1 || { tail -20 "$O/bench_kt8.log"; exit 1; }
step done
