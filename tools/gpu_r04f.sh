#!/bin/bash
# round 4: select v2 phases, the shard step, kernel-10 append ablation (MODE 4096) and slow-path priority
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 120 python -u tools/debug_sharded_ties.py > $O/ties.log 2>&1 || { tail -30 $O/ties.log; exit 1; }
tail -2 $O/ties.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
timeout -k 10 300 python -u tools/select_phases.py > $O/select_phases_cfg3.json 2>&1 || { tail -20 $O/select_phases_cfg3.json; exit 1; }
grep -A 16 median_rep $O/select_phases_shard.json $O/select_phases_cfg3.json | tr -d ' \n'; echo
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 800000,804096,804128,800032 --rounds 8 --burst 100 > $O/k10_shard_app.txt 2>&1 || { tail -20 $O/k10_shard_app.txt; exit 1; }
grep -h "slow_path\|min" $O/k10_shard_app.txt
timeout -k 10 300 python -u tools/k10_variants.py --variants 800000,804096,804128,800032 --rounds 6 > $O/k10_10m_app.txt 2>&1 || { tail -20 $O/k10_10m_app.txt; exit 1; }
grep -h "slow_path\|min" $O/k10_10m_app.txt
