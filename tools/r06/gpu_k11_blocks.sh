#!/bin/bash
# Round 6: kernel 11 with kept scores (up to 4 chunks, <= 256 rows per wave): its tests, then config 2 at
# 250 (the plan) / 192 / 160 / 128 workgroups (RFX_VALU_BLOCKS), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06kb}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"))'
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen_valu.py tests/test_gpu_sharded.py tests/test_gpu_filters.py tests/test_gpu_union.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -1 $O/pytest_k11.log
for i in 1 2; do for nb in 250 192 160 128; do
  RFX_VALU_BLOCKS=$nb timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/cfg2_b${nb}_$i.log 2>&1 || { tail -20 $O/cfg2_b${nb}_$i.log; exit 1; }
  echo -n "blocks=$nb $i: "; python3 -c "$S" < $O/cfg2_b${nb}_$i.log
done; done
