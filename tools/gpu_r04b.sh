#!/bin/bash
# round 4: the new GPU tests (gathered merge kernel, records pack of the one-launch searches, the
# two-pass scan behind the sharded store, the int8-copy capacity guard), then the shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_merge.py tests/test_gpu_screen_capacity.py tests/test_gpu_sharded.py tests/test_gpu_screen_valu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log
