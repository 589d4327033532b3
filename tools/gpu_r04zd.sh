#!/bin/bash
# round 4 final build: rocprofv3 kernel trace of config 2 (kernel 11 with its fallback inside the launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04zd; mkdir -p $O
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 300 --warmup 20 --event-stride 16 --no-cpu-baseline"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt2 -- python $R/bench.py $C2 > $O/bench_kt2.log 2>&1 || { tail -20 $O/bench_kt2.log; exit 1; }
python3 -c "
import csv
r=list(csv.DictReader(open('$O/kt2/kt2_kernel_stats.csv')))
for x in r[:6]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,2))
"
