#!/bin/bash
# round 4: DPP wave reductions (no ds_bpermute) in kernel 11, the query quantiser and the select's
# re-score: kernel 11 phases + config 2, the two-pass tests, the shard step and config 3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
cat $O/k11_phases.json | tr -d ' \n'; echo
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
tail -1 $O/bench_cfg2.log | python3 -c "$S"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen_valu.py tests/test_gpu_screen.py tests/test_gpu_sharded.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
