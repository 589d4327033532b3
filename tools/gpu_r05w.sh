#!/bin/bash
# round 5 final evidence on the shipped build (kernel 11 early re-score; debug counters of missing keys): smoke, the default bench, the
# 8-GPU shard step and config 2 (same box), rocprofv3 kernel-trace summaries, and PMC FETCH_SIZE /
# WRITE_SIZE passes (one counter per pass) of kernels 10 and 11 for profiles/pmc_traffic.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["roofline"].get("traffic"), d.get("oracle_check", {}).get("ok"), d.get("build_id"))'
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
python3 -c "$S" < $O/bench_default.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
python3 -c "$S" < $O/bench_shard_fc.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg3_b.log 2>&1 || { tail -30 $O/bench_cfg3_b.log; exit 1; }
python3 -c "$S" < $O/bench_cfg3_b.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc_b.log 2>&1 || { tail -30 $O/bench_shard_fc_b.log; exit 1; }
python3 -c "$S" < $O/bench_shard_fc_b.log
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
python3 -c "$S" < $O/bench_cfg2.log
cd /tmp
C3="--steps 10 --warmup 2 --no-cpu-baseline"
CS="--rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline"
C2="--rows 100000 --dtype f32 --nq 1 --steps 300 --warmup 20 --event-stride 16 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3 -o kt3 -- python $R/bench.py $C3 > $O/bench_kt3.log 2>&1 || { tail -20 $O/bench_kt3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kts -o kts -- python $R/bench.py $CS > $O/bench_kts.log 2>&1 || { tail -20 $O/bench_kts.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt2 -- python $R/bench.py $C2 > $O/bench_kt2.log 2>&1 || { tail -20 $O/bench_kt2.log; exit 1; }
P3="--steps 4 --warmup 1 --no-cpu-baseline --oracle-stride 0"
Ps="--rows 1250000 --force-comm --steps 20 --warmup 2 --no-cpu-baseline --oracle-stride 0"
P2="--rows 100000 --dtype f32 --nq 1 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0"
for c in 3 s 2; do
  eval P=\$P$c
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf$c -o pmcf$c -- python $R/bench.py $P > $O/bench_pmcf$c.log 2>&1 || { tail -20 $O/bench_pmcf$c.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw$c -o pmcw$c -- python $R/bench.py $P > $O/bench_pmcw$c.log 2>&1 || { tail -20 $O/bench_pmcw$c.log; exit 1; }
done
find $O -name "*.csv" | head -40
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -60 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
timeout -k 10 300 python -u tools/k11_phases.py --reps 160 > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
grep -v amdgpu $O/k11_phases.json | tr -d '\n '; echo
