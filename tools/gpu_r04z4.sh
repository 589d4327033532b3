#!/bin/bash
# round 4: select re-score with 192 rows per round (one round for nearly every query): tests, select
# phases at the shard and at 10M, the shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z4; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_sharded.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
grep -v amdgpu $O/select_phases_shard.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['survivors_mean'], d['median_rep'])"
timeout -k 10 300 python -u tools/select_phases.py > $O/select_phases_10m.json 2>&1 || { tail -20 $O/select_phases_10m.json; exit 1; }
grep -v amdgpu $O/select_phases_10m.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['survivors_mean'], d['median_rep'])"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
