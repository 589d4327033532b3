#!/bin/bash
# round 4 closing measurements on the final build: config 2, config 3 (default run), the 8-GPU shard
# step (1-rank RCCL), config 4's shard (12.5M x 1024 f16, two-pass, XCD-balanced kernel 10)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z5; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d["phases_ms"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check",{}).get("ok"), d["build_id"])'
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
tail -1 $O/bench_cfg2.log | python3 -c "$S"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
timeout -k 10 500 python -u bench.py > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
timeout -k 10 600 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_cfg4_shard.log 2>&1 || { tail -30 $O/bench_cfg4_shard.log; exit 1; }
tail -1 $O/bench_cfg4_shard.log | python3 -c "$S"
