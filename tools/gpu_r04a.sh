#!/bin/bash
# round 4, first call: default bench (config 3), the 8-GPU shard step through a 1-rank RCCL
# communicator, and kernel 10's MODE 16 warm-up ablation (built in round 3, never measured)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 420 python -u bench.py > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 8032,8048,8000,8016 --rounds 8 --burst 100 > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -h "slow_path\|min" $O/k10_shard.txt
