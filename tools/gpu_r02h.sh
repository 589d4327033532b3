#!/bin/bash
# Round-2 GPU session H (final evidence of the round's library): smoke, the -m gpu suite, the
# default bench (config 3) with kernel stats, config 2 with kernel stats and PMC traffic, the N > 1
# rehearsal on one GPU.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-r02h}"
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
step rehearsal
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --one-device --check --no-cpu-baseline "$@" >> "$O/rehearsal.log" 2>&1
}
run 2 --rows 1000000 --steps 5 --warmup 2 && run 4 --rows 1000003 --steps 5 --warmup 2 && \
  run 2 --rows 200000 --dim 1024 --dtype f16 --steps 5 --warmup 2 || { tail -40 "$O/rehearsal.log"; exit 1; }
grep -E "check ok" "$O/rehearsal.log"
cd /tmp && export TMPDIR=/tmp
step kt3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt3" -o kt3 -- python "$R/bench.py" --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt3.log" 2>&1 || { tail -20 "$O/bench_kt3.log"; exit 1; }
step kt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt2 -- python "$R/bench.py" $C2 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt2.log" 2>&1 || { tail -20 "$O/bench_kt2.log"; exit 1; }
step pmc2
P2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 50 --warmup 10 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf2" -o pmcf2 -- python "$R/bench.py" $P2 > "$O/bench_pmcf2.log" 2>&1 || { tail -20 "$O/bench_pmcf2.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmcw2" -o pmcw2 -- python "$R/bench.py" $P2 > "$O/bench_pmcw2.log" 2>&1 || { tail -20 "$O/bench_pmcw2.log"; exit 1; }
step done
