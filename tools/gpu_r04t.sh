#!/bin/bash
# round 4: select a_k back to the count (16-B LDS reads); kernel 11's LB by the same count: tests,
# select phases at the shard, kernel 11 phases, config 2, the shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_screen_valu.py tests/test_gpu_sharded.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
grep -v amdgpu $O/select_phases_shard.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['median_rep'])"
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
grep -v amdgpu $O/k11_phases.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['median'])"
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
tail -1 $O/bench_cfg2.log | python3 -c "$S"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
