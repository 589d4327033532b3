#!/bin/bash
# round 3: config 5 through an RFX_INDEX=ivf store; HBM traffic (PMC FETCH_SIZE / WRITE_SIZE passes)
# of kernel 11 at config 2 and kernel 10 at config 4's shard
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ivf_cfg5.py -x -v -s --timeout 800 --timeout-method thread > $O/pytest_cfg5.log 2>&1 || { tail -30 $O/pytest_cfg5.log; exit 1; }
grep -E "recall|passed|failed" $O/pytest_cfg5.log
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
C4="--rows 12500000 --dim 1024 --dtype f16 --steps 5 --warmup 1 --no-cpu-baseline --oracle-stride 0"
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf2 -o pmcf2 -- python $R/bench.py $C2 > $O/bench_pmcf2.log 2>&1 || { tail -20 $O/bench_pmcf2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw2 -o pmcw2 -- python $R/bench.py $C2 > $O/bench_pmcw2.log 2>&1 || { tail -20 $O/bench_pmcw2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf4 -o pmcf4 -- python $R/bench.py $C4 > $O/bench_pmcf4.log 2>&1 || { tail -20 $O/bench_pmcf4.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw4 -o pmcw4 -- python $R/bench.py $C4 > $O/bench_pmcw4.log 2>&1 || { tail -20 $O/bench_pmcw4.log; exit 1; }
find $O -name "*.csv" | head -20
