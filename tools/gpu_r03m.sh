#!/bin/bash
# round 3: kernel 10 with alternating accumulators (deferred epilogue) against the in-place epilogue;
# one-launch multi-store union tests + rocprof launch counts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_union.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/k10_variants.py --variants 832,800,928,801,929 --rounds 4 > $O/variants.json 2> $O/variants.err || { tail -5 $O/variants.err; exit 1; }
cat $O/variants.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -c 2500 $O/bench_cfg3.log
for m in union per-store; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python -u tools/union_launches.py --mode $m > $O/union_$m.log 2>&1 || { tail -20 $O/union_$m.log; exit 1; }
  tail -1 $O/union_$m.log
  find $O/prof_$m -name "*kernel_stats.csv" -exec grep -h "scan\|merge" {} \; | cut -c1-160
done
