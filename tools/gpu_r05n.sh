#!/bin/bash
# round 5 extra evidence on the shipped build: the union-while-question test, config 4's shard, config 5's
# IVF shard, and the N = 2 / 4 rehearsals (ranks sharing the GPU, gloo exchange, rank-0 oracle check)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"), d.get("build_id"))'
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_union.py > $O/pytest_union.log 2>&1 || { tail -40 $O/pytest_union.log; exit 1; }
tail -2 $O/pytest_union.log
timeout -k 10 400 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 20 --warmup 3 --oracle-stride 4 > $O/bench_cfg4_shard.log 2>&1 || { tail -20 $O/bench_cfg4_shard.log; exit 1; }
python3 -c "$S" < $O/bench_cfg4_shard.log
timeout -k 10 400 python -u tools/bench_ivf.py > $O/ivf_bench.log 2>&1 || { tail -20 $O/ivf_bench.log; exit 1; }
tail -3 $O/ivf_bench.log | cut -c1-400
run() {
  local n=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --one-device --check --no-cpu-baseline "$@"
}
run 2 --rows 1000000 --steps 5 --warmup 2 > $O/rehearsal2.log 2>&1 || { tail -30 $O/rehearsal2.log; exit 1; }
tail -1 $O/rehearsal2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['oracle_check']['ok'], d['oracle_check'].get('rows_identical_frac'))"
run 4 --rows 1000003 --steps 5 --warmup 2 > $O/rehearsal4.log 2>&1 || { tail -30 $O/rehearsal4.log; exit 1; }
tail -1 $O/rehearsal4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['oracle_check']['ok'], d['oracle_check'].get('rows_identical_frac'))"
