#!/bin/bash
# round 4: branch-free key ranks in the select and kernel 11: their tests, the shard step, config 2,
# select phases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_screen_valu.py tests/test_gpu_sharded.py tests/test_gpu_merge.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard', d['ms_per_step'], d['phases_ms'])"
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
tail -1 $O/bench_cfg2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
grep -A 16 median_rep $O/select_phases_shard.json | tr -d ' \n'; echo
