#!/bin/bash
# Round 6: the select with the exact fallback inside its launch (k_select_fb.h).  The two-pass GPU tests
# (forced and natural fallbacks, masks, records, shards), then the default (one launch) against
# RFX_SELECT_FB=0 (select + gated kernel 6 + gated merge), interleaved: the 8-GPU shard and config 3; a
# rocprof kernel-trace of the shard step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/${1:-gpurun_out/r06b}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"))'
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_screen_w2.py tests/test_gpu_filters.py tests/test_gpu_sharded.py tests/test_gpu_screen_capacity.py tests/test_gpu_bench_rehearsal.py tests/test_dist_gpu.py tests/test_gpu_union.py > $O/pytest_selfb.log 2>&1 || { tail -40 $O/pytest_selfb.log; exit 1; }
tail -1 $O/pytest_selfb.log
for i in 1 2; do
  for v in 1 0; do
    RFX_SELECT_FB=$v timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/shard_fb${v}_$i.log 2>&1 || { tail -20 $O/shard_fb${v}_$i.log; exit 1; }
    echo -n "shard fb=$v $i: "; python3 -c "$S" < $O/shard_fb${v}_$i.log
    RFX_SELECT_FB=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/cfg3_fb${v}_$i.log 2>&1 || { tail -20 $O/cfg3_fb${v}_$i.log; exit 1; }
    echo -n "cfg3 fb=$v $i: "; python3 -c "$S" < $O/cfg3_fb${v}_$i.log
  done
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktS -o ktS -- python $R/bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_ktS.log 2>&1 || { tail -20 $O/bench_ktS.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/ktS/ktS_kernel_stats.csv')):
    print(r['Calls'], round(float(r['AverageNs'])/1000,2), r['Name'][:90])
"
