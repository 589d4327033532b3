#!/bin/bash
# round 4: tie debugging of the screened sharded store, union tests, shard step, select phases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 300 python -u tools/debug_sharded_ties.py > $O/ties.log 2>&1 || { tail -30 $O/ties.log; exit 1; }
cat $O/ties.log
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_union.py > $O/pytest_union.log 2>&1 || { tail -40 $O/pytest_union.log; exit 1; }
grep -h "union of\|passed\|failed" $O/pytest_union.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log
timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/select_phases_shard.json 2>&1 || { tail -20 $O/select_phases_shard.json; exit 1; }
timeout -k 10 300 python -u tools/select_phases.py > $O/select_phases_cfg3.json 2>&1 || { tail -20 $O/select_phases_cfg3.json; exit 1; }
cat $O/select_phases_shard.json $O/select_phases_cfg3.json
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 800000,800032,802048,802080 --rounds 8 --burst 100 > $O/k10_shard_prio.txt 2>&1 || { tail -20 $O/k10_shard_prio.txt; exit 1; }
grep -h "slow_path\|min" $O/k10_shard_prio.txt
