#!/bin/bash
# round 4: the select kernel's a_k by wave top-k (DPP) instead of the O(n_c^2) count: the two-pass
# tests (incl. the full-size 10M check), select phases at the shard, the shard step and config 3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py tests/test_gpu_screen_capacity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
grep -v amdgpu $O/select_phases_shard.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['median_rep'])"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
