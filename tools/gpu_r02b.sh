#!/bin/bash
# Round-2 GPU session B: the whole -m gpu suite (incl. full-size parity, store, sharded, RCCL) and
# the N>1 bench rehearsal on one GPU (gloo exchange, --check vs a whole-index search).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02b"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
echo "== pytest $(date +%T)"
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=8 -v --timeout 420 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
echo "== rehearsal $(date +%T)"
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --one-device --check --no-cpu-baseline "$@" >> "$O/rehearsal.log" 2>&1
}
run 2 --rows 1000000 --steps 5 --warmup 2 && run 4 --rows 1000003 --steps 5 --warmup 2 || { tail -40 "$O/rehearsal.log"; exit 1; }
grep -E "check ok|\"value\"" "$O/rehearsal.log" | cut -c1-160
echo "== done $(date +%T)"
