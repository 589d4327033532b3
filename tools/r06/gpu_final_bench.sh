#!/bin/bash
# Round 6 evidence on one box, one call: smoke, the default bench (config 3), the 8-GPU shard step, config 2,
# the micro-batch sizes (10M bf16 nq 32, 100k f32 nq 32), rocprofv3 kernel-trace summaries of them and PMC
# FETCH_SIZE / WRITE_SIZE passes (one counter per pass) of kernels 10 (8- and 2-wave) and 11.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/${1:-gpurun_out/r06f}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["config"].get("nq"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["roofline"].get("traffic"), d.get("oracle_check", {}).get("ok"), d.get("build_id"))'
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
python3 -c "$S" < $O/bench_default.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
python3 -c "$S" < $O/bench_shard_fc.log
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
python3 -c "$S" < $O/bench_cfg2.log
timeout -k 10 300 python -u bench.py --nq 32 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_10m_nq32.log 2>&1 || { tail -30 $O/bench_10m_nq32.log; exit 1; }
python3 -c "$S" < $O/bench_10m_nq32.log
timeout -k 10 300 python -u bench.py --nq 32 --scan exact --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_10m_nq32_exact.log 2>&1 || { tail -30 $O/bench_10m_nq32_exact.log; exit 1; }
python3 -c "$S" < $O/bench_10m_nq32_exact.log
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 32 --steps 300 --warmup 30 --no-cpu-baseline > $O/bench_100k_f32_nq32.log 2>&1 || { tail -30 $O/bench_100k_f32_nq32.log; exit 1; }
python3 -c "$S" < $O/bench_100k_f32_nq32.log
cd /tmp
C3="--steps 10 --warmup 2 --no-cpu-baseline"
CS="--rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline"
C2="--rows 100000 --dtype f32 --nq 1 --steps 300 --warmup 20 --event-stride 16 --no-cpu-baseline"
CQ="--nq 32 --steps 10 --warmup 2 --no-cpu-baseline"
for c in 3 S 2 Q; do
  eval C=\$C$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$c -o kt$c -- python $R/bench.py $C > $O/bench_kt$c.log 2>&1 || { tail -20 $O/bench_kt$c.log; exit 1; }
done
P3="--steps 4 --warmup 1 --no-cpu-baseline --oracle-stride 0"
PS="--rows 1250000 --force-comm --steps 20 --warmup 2 --no-cpu-baseline --oracle-stride 0"
P2="--rows 100000 --dtype f32 --nq 1 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
PQ="--nq 32 --steps 4 --warmup 1 --no-cpu-baseline --oracle-stride 0"
for c in 3 S 2 Q; do
  eval P=\$P$c
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf$c -o pmcf$c -- python $R/bench.py $P > $O/bench_pmcf$c.log 2>&1 || { tail -20 $O/bench_pmcf$c.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw$c -o pmcw$c -- python $R/bench.py $P > $O/bench_pmcw$c.log 2>&1 || { tail -20 $O/bench_pmcw$c.log; exit 1; }
done
find $O -name "*.csv" | head -60
