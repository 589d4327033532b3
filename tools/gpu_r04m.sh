#!/bin/bash
# round 4: config 4 — the whole 100M x 1024 f16 corpus on one GPU (the int8 copy does not fit beside
# 204.8 GB of rows: the capacity guard sends --scan auto to the exact kernel 8) and the 12.5M-row
# shard of the 8-GPU run (two-pass, oracle-checked)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:40], d["value"], d["ms_per_step"], d["config"]["scan_kernel"][:160], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 600 python -u bench.py --rows 100000000 --dim 1024 --dtype f16 --steps 10 --warmup 2 --oracle-stride 0 --no-cpu-baseline > $O/bench_cfg4_whole.log 2>&1 || { tail -30 $O/bench_cfg4_whole.log; exit 1; }
tail -1 $O/bench_cfg4_whole.log | python3 -c "$S"
timeout -k 10 420 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline > $O/bench_cfg4_shard.log 2>&1 || { tail -30 $O/bench_cfg4_shard.log; exit 1; }
tail -1 $O/bench_cfg4_shard.log | python3 -c "$S"
