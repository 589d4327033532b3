#!/bin/bash
# Round 6: kernel 10 started from the quantiser's seed bound (default) against no seed (RFX_K10_SEED=0), config 3
# and the 8-GPU shard, interleaved on one box; then the two-pass tests on the seeded build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06s}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"))'
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_screen_w2.py tests/test_gpu_filters.py tests/test_gpu_sharded.py tests/test_gpu_screen_capacity.py > $O/pytest_seed.log 2>&1 || { tail -40 $O/pytest_seed.log; exit 1; }
tail -1 $O/pytest_seed.log
for i in 1 2; do
  for sd in 1 0; do
    RFX_K10_SEED=$sd timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/shard_seed${sd}_$i.log 2>&1 || { tail -20 $O/shard_seed${sd}_$i.log; exit 1; }
    echo -n "shard seed=$sd $i: "; python3 -c "$S" < $O/shard_seed${sd}_$i.log
    RFX_K10_SEED=$sd timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/cfg3_seed${sd}_$i.log 2>&1 || { tail -20 $O/cfg3_seed${sd}_$i.log; exit 1; }
    echo -n "cfg3 seed=$sd $i: "; python3 -c "$S" < $O/cfg3_seed${sd}_$i.log
  done
done
