#!/bin/bash
# round 4: capacity guard, sharded two-pass, incremental union (+ byte budget), then the shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_screen_capacity.py tests/test_gpu_sharded.py tests/test_gpu_union.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -h "union of\|passed\|failed" $O/pytest.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
timeout -k 10 300 python -u tools/select_phases.py > $O/select_phases_cfg3.json 2>&1 || { tail -20 $O/select_phases_cfg3.json; exit 1; }
cat $O/select_phases_shard.json $O/select_phases_cfg3.json
