#!/bin/bash
# round 4 final evidence on the XCD-balanced build: rocprofv3 kernel-trace summaries (config 3, the
# 8-GPU shard step through a 1-rank RCCL communicator, config 2), PMC traffic of kernel 10 (config 3
# and the shard) and kernel 11 (config 2) in separate FETCH_SIZE / WRITE_SIZE passes, and the N = 2 / 4
# rehearsals (ranks sharing the GPU, gloo exchange) with the rank-0 oracle check
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z2; mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --one-device --check --no-cpu-baseline "$@"
}
run 2 --rows 1000000 --steps 5 --warmup 2 > $O/rehearsal2.log 2>&1 || { tail -30 $O/rehearsal2.log; exit 1; }
tail -1 $O/rehearsal2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['oracle_check']['ok'], d['oracle_check']['rows_identical_frac'])"
run 4 --rows 1000003 --steps 5 --warmup 2 > $O/rehearsal4.log 2>&1 || { tail -30 $O/rehearsal4.log; exit 1; }
tail -1 $O/rehearsal4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['oracle_check']['ok'], d['oracle_check']['rows_identical_frac'])"
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 300 --warmup 20 --event-stride 16 --no-cpu-baseline"
C3="--steps 20 --warmup 3 --no-cpu-baseline"
CS="--rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3 -o kt3 -- python $R/bench.py $C3 > $O/bench_kt3.log 2>&1 || { tail -20 $O/bench_kt3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kts -o kts -- python $R/bench.py $CS > $O/bench_kts.log 2>&1 || { tail -20 $O/bench_kts.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt2 -- python $R/bench.py $C2 > $O/bench_kt2.log 2>&1 || { tail -20 $O/bench_kt2.log; exit 1; }
P2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
P3="--steps 6 --warmup 3 --no-cpu-baseline --oracle-stride 0"
PS="--rows 1250000 --force-comm --steps 20 --warmup 10 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf2 -o pmcf2 -- python $R/bench.py $P2 > $O/bench_pmcf2.log 2>&1 || { tail -20 $O/bench_pmcf2.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw2 -o pmcw2 -- python $R/bench.py $P2 > $O/bench_pmcw2.log 2>&1 || { tail -20 $O/bench_pmcw2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf3 -o pmcf3 -- python $R/bench.py $P3 > $O/bench_pmcf3.log 2>&1 || { tail -20 $O/bench_pmcf3.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw3 -o pmcw3 -- python $R/bench.py $P3 > $O/bench_pmcw3.log 2>&1 || { tail -20 $O/bench_pmcw3.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcfs -o pmcfs -- python $R/bench.py $PS > $O/bench_pmcfs.log 2>&1 || { tail -20 $O/bench_pmcfs.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcws -o pmcws -- python $R/bench.py $PS > $O/bench_pmcws.log 2>&1 || { tail -20 $O/bench_pmcws.log; exit 1; }
ls $O
