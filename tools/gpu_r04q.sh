#!/bin/bash
# round 4 evidence: the N>1 rehearsal with the rank-0 oracle check of the gathered answer; rocprofv3
# kernel-trace summaries of config 3, the 8-GPU shard step (1-rank RCCL) and config 2; PMC traffic of
# kernels 10 and 11 (separate FETCH_SIZE / WRITE_SIZE passes); the union-follow timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q; mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --one-device --check --no-cpu-baseline "$@"
}
run 2 --rows 1000000 --steps 5 --warmup 2 > $O/rehearsal2_cfg3shape.log 2>&1 || { tail -30 $O/rehearsal2_cfg3shape.log; exit 1; }
grep -E "^check|oracle_check" $O/rehearsal2_cfg3shape.log | python3 -c "import sys; [print(l.strip()[:120]) for l in sys.stdin]"
tail -1 $O/rehearsal2_cfg3shape.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['oracle_check'])"
run 2 --rows 100000 --nq 1 --dtype f32 --steps 20 --warmup 2 > $O/rehearsal2_cfg2shape.log 2>&1 || { tail -30 $O/rehearsal2_cfg2shape.log; exit 1; }
tail -1 $O/rehearsal2_cfg2shape.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['oracle_check'])"
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_union.py > $O/pytest_union.log 2>&1 || { tail -30 $O/pytest_union.log; exit 1; }
grep -E "union of|passed|failed" $O/pytest_union.log
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 300 --warmup 20 --event-stride 16 --no-cpu-baseline"
C3="--steps 20 --warmup 3 --no-cpu-baseline"
CS="--rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3 -o kt3 -- python $R/bench.py $C3 > $O/bench_kt3.log 2>&1 || { tail -20 $O/bench_kt3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kts -o kts -- python $R/bench.py $CS > $O/bench_kts.log 2>&1 || { tail -20 $O/bench_kts.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt2 -- python $R/bench.py $C2 > $O/bench_kt2.log 2>&1 || { tail -20 $O/bench_kt2.log; exit 1; }
P2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
P3="--steps 4 --warmup 1 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf2 -o pmcf2 -- python $R/bench.py $P2 > $O/bench_pmcf2.log 2>&1 || { tail -20 $O/bench_pmcf2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw2 -o pmcw2 -- python $R/bench.py $P2 > $O/bench_pmcw2.log 2>&1 || { tail -20 $O/bench_pmcw2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf3 -o pmcf3 -- python $R/bench.py $P3 > $O/bench_pmcf3.log 2>&1 || { tail -20 $O/bench_pmcf3.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw3 -o pmcw3 -- python $R/bench.py $P3 > $O/bench_pmcw3.log 2>&1 || { tail -20 $O/bench_pmcw3.log; exit 1; }
find $O -name "*.csv" | head -30
