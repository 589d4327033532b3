#!/bin/bash
# round 3: config 3's 8-GPU shard (1.25M rows) on one GPU — plain and through the 1-rank RCCL step
# (--force-comm: records, gather, gathered merge), with rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03w; mkdir -p $O
S="--rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
timeout -k 10 200 python -u bench.py $S > $O/bench_shard.log 2>&1 || { tail -20 $O/bench_shard.log; exit 1; }
timeout -k 10 200 python -u bench.py $S --force-comm > $O/bench_shard_fc.log 2>&1 || { tail -20 $O/bench_shard_fc.log; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python $R/bench.py $S --force-comm > $O/bench_shard_fc_prof.log 2>&1 || { tail -20 $O/bench_shard_fc_prof.log; exit 1; }
for f in $O/bench_shard.log $O/bench_shard_fc.log; do tail -c 1200 $f; echo; done
find $O/kt -name "*stats*.csv" | head
