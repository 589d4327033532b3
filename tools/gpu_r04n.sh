#!/bin/bash
# round 4: the pipelined N > 1 step (two CU-masked streams) at the 8-GPU shard through a 1-rank RCCL
# communicator, against the sequential step; then kernel 11 / config 4 (r04l, r04m)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"], d.get("oracle_check",{}).get("ok"), d["config"].get("pipeline") is not None)'
for pl in on off on; do
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline --pipeline $pl > $O/bench_shard_pipe_$pl.log 2>&1 || { tail -30 $O/bench_shard_pipe_$pl.log; exit 1; }
tail -1 $O/bench_shard_pipe_$pl.log | python3 -c "$S"
done
bash tools/gpu_r04l.sh && bash tools/gpu_r04m.sh
