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
for v in 800 928 801 809; do
  timeout -k 10 120 python -u tools/k10_variants.py --variants $v --seconds 16 > $O/pw_run_$v.json 2> $O/pw_run_$v.err &
  pid=$!
  sleep 12
  for i in 1 2 3; do timeout -k 5 20 rocm-smi --showclocks --showpower >> $O/pw_smi_$v.txt 2>&1; sleep 0.5; done
  wait $pid || { echo "run $v failed"; tail -5 $O/pw_run_$v.err; exit 1; }
  echo "$v $(cat $O/pw_run_$v.json) | $(grep -oE 'sclk clock level: [0-9]+: \([0-9]+Mhz\)|Power \(W\): [0-9.]+' $O/pw_smi_$v.txt | tr '\n' ' ')"
done
P3="--steps 5 --warmup 1 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf3 -o pmcf3 -- python bench.py $P3 > $O/bench_pmcf3.log 2>&1 || { tail -20 $O/bench_pmcf3.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw3 -o pmcw3 -- python bench.py $P3 > $O/bench_pmcw3.log 2>&1 || { tail -20 $O/bench_pmcw3.log; exit 1; }
find $O/pmcf3 $O/pmcw3 -name "*.csv" | head
