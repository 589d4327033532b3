#!/bin/bash
# Round 6: kernel 11 with 2 / 4 query slots for small batches against the previous build (librfx_base.so):
# kernel 11's tests, then 100k x 768 f32 at nq 2 / 3 / 4 / 8, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06nq}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"))'
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen_valu.py tests/test_gpu_screen.py tests/test_gpu_sharded.py tests/test_gpu_filters.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -1 $O/pytest_k11.log
for i in 1 2; do for nq in 2 3 4 8; do
  timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq $nq --steps 1000 --warmup 100 --event-stride 16 --no-cpu-baseline > $O/nq${nq}_new_$i.log 2>&1 || { tail -20 $O/nq${nq}_new_$i.log; exit 1; }
  echo -n "nq=$nq new $i: "; python3 -c "$S" < $O/nq${nq}_new_$i.log
  RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq $nq --steps 1000 --warmup 100 --event-stride 16 --no-cpu-baseline > $O/nq${nq}_base_$i.log 2>&1 || { tail -20 $O/nq${nq}_base_$i.log; exit 1; }
  echo -n "nq=$nq base $i: "; python3 -c "$S" < $O/nq${nq}_base_$i.log
done; done
