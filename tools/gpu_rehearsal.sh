#!/bin/bash
# N>1 path rehearsal on one GPU: gloo exchange, every rank on cuda:0, --check = sharded top-k
# equals one whole-index search.  Config-3 shape at 1M rows (2 and 4 ranks), config-2 shape (2 ranks).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
export PYTHONDONTWRITEBYTECODE=1
: > "$O/rehearsal.log"
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --one-device --check --no-cpu-baseline "$@" \
    >> "$O/rehearsal.log" 2>&1
}
run 2 --rows 1000000 --steps 5 --warmup 2 && run 4 --rows 1000003 --steps 5 --warmup 2 && \
  run 2 --rows 100000 --nq 1 --dtype f32 --steps 20 --warmup 2 || { echo "rehearsal rc=$?"; tail -30 "$O/rehearsal.log"; exit 1; }
grep -E "check|value" "$O/rehearsal.log" | cut -c1-200
