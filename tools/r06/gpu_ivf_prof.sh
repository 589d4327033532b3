#!/bin/bash
# Round 6: rocprofv3 kernel-trace summary of config 5 (tools/bench_ivf.py) on the current build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/${1:-gpurun_out/r06ivfp}; mkdir -p $O
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python $R/tools/bench_ivf.py > $O/ivf_bench_kt.log 2>&1 || { tail -20 $O/ivf_bench_kt.log; exit 1; }
cp $O/kt/kt_kernel_stats.csv $O/ivf_kernel_stats.csv
python3 -c "import csv,sys; [print(r[0][:70], r[1], r[2], r[3]) for r in list(csv.reader(open(sys.argv[1])))[:16]]" $O/ivf_kernel_stats.csv
tail -1 $O/ivf_bench_kt.log | cut -c1-200
