#!/bin/bash
# Round-2 GPU session E: smoke, the N > 1 bench rehearsal on one GPU (gloo exchange between ranks
# sharing cuda:0, --check against a whole-index search), the config-5 IVF bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02e"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
echo "== rehearsal $(date +%T)"
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --one-device --check --no-cpu-baseline "$@" >> "$O/rehearsal.log" 2>&1
}
run 2 --rows 1000000 --steps 5 --warmup 2 && run 4 --rows 1000003 --steps 5 --warmup 2 && \
  run 2 --rows 100000 --dim 768 --dtype f32 --nq 1 --steps 20 --warmup 5 || { tail -40 "$O/rehearsal.log"; exit 1; }
grep -E "check ok|\"value\"" "$O/rehearsal.log" | cut -c1-160
echo "== ivf $(date +%T)"
timeout -k 10 400 python -u tools/bench_ivf.py > "$O/ivf.log" 2>&1 || { tail -20 "$O/ivf.log"; exit 1; }
tail -1 "$O/ivf.log" | cut -c1-400
echo "== done $(date +%T)"
