#!/bin/bash
# Round-2 GPU session F (fresh container, library rebuilt): smoke, the -m gpu suite, the default
# bench (config 3) with kernel stats, the N > 1 rehearsal on one GPU and the config-5 IVF bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02f"
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
step rehearsal
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --one-device --check --no-cpu-baseline "$@" >> "$O/rehearsal.log" 2>&1
}
run 2 --rows 1000000 --steps 5 --warmup 2 && run 4 --rows 1000003 --steps 5 --warmup 2 && \
  run 2 --rows 100000 --dim 768 --dtype f32 --nq 1 --steps 20 --warmup 5 || { tail -40 "$O/rehearsal.log"; exit 1; }
grep -E "check ok|\"value\"" "$O/rehearsal.log" | cut -c1-160
step ivf
timeout -k 10 400 python -u tools/bench_ivf.py > "$O/ivf.log" 2>&1 || { tail -20 "$O/ivf.log"; exit 1; }
tail -1 "$O/ivf.log" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
step kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt3" -o kt3 -- python "$R/bench.py" --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt3.log" 2>&1 || { tail -20 "$O/bench_kt3.log"; exit 1; }
step done
