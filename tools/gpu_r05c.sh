#!/bin/bash
# round 5: kernel 10's new fold and the one-barrier-per-tile schedule (debug TB, RING 12) (u32-score lists, integer pass threshold, per-position inserts in the first
# tiles) against round 4's (debug kModeFold1); config 3 and the 8-GPU shard step; the one-call sharded
# search's host issue; the round-5 GPU tests (score rule, dropped copies, unions, sharded C path, full size)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("phases_ms"), d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check",{}).get("ok"), d["two_pass"]["survivors_mean"] if "two_pass" in d else "", d["build_id"])'
V=80000000,81048576,80524288,120000000,122097152,122621440
timeout -k 10 400 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -v amdgpu $O/k10_shard.txt | python3 -c "import sys,json; t=sys.stdin.read(); i=t.rfind('{\n'); d=json.loads(t[i:]); print({k:v['ms_per_launch_min'] for k,v in d['variants'].items()})"
timeout -k 10 400 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
grep -v amdgpu $O/k10_10m.txt | python3 -c "import sys,json; t=sys.stdin.read(); i=t.rfind('{\n'); d=json.loads(t[i:]); print({k:v['ms_per_launch_min'] for k,v in d['variants'].items()})"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline --pipeline on --reserve-cus 0 > $O/bench_shard_fc_pipe0.log 2>&1 || { tail -30 $O/bench_shard_fc_pipe0.log; exit 1; }
tail -1 $O/bench_shard_fc_pipe0.log | python3 -c "$S"
timeout -k 10 300 python -u tools/k10_trips.py > $O/k10_trips_prod.json 2>&1 || { tail -20 $O/k10_trips_prod.json; exit 1; }
timeout -k 10 300 python -u tools/k10_trips.py --variant 122105344 > $O/k10_trips_tb.json 2>&1 || { tail -20 $O/k10_trips_tb.json; exit 1; }
grep -h "total" $O/k10_trips_prod.json $O/k10_trips_tb.json
timeout -k 10 1200 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_screen_capacity.py tests/test_gpu_union.py tests/test_gpu_sharded.py tests/test_gpu_fused.py tests/test_gpu_filters.py tests/test_gpu_merge.py tests/test_gpu_parity.py tests/test_gpu_screen_valu.py tests/test_gpu_fullsize.py tests/test_gpu_bench_rehearsal.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u tools/sharded_host_issue.py > $O/sharded_host_issue.json 2>&1 || { tail -20 $O/sharded_host_issue.json; exit 1; }
grep -v amdgpu $O/sharded_host_issue.json
