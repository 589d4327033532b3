#!/bin/bash
# Round-2 GPU session N (final library, kernel 6 and kernel 8 with 4-slot rings): smoke, the -m gpu
# suite, the default bench (config 3, oracle-checked), a ring-3 side build of kernel 6 alternating
# with production, the 8-GPU shard shape, kernel stats and PMC traffic of config 3.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-r02n}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('oracle_check', {}).get('ok'))" "$1" "$2"; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
step pytest
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=8 -q --timeout 420 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
step bench
timeout -k 10 400 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
show "$O/bench.log" cfg3
step ring3
C3="--no-cpu-baseline --steps 40 --warmup 5 --oracle-stride 0"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $C3 > "$O/prod_$i.log" 2>&1 || { tail -20 "$O/prod_$i.log"; exit 1; }
  show "$O/prod_$i.log" prod_$i
  RFX_LIB="$R/rag-foundation_amd/rfx/librfx_k6r3.so" timeout -k 10 200 python -u bench.py $C3 > "$O/k6r3_$i.log" 2>&1 || { tail -20 "$O/k6r3_$i.log"; exit 1; }
  show "$O/k6r3_$i.log" k6r3_$i
done
step shard
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 16 > "$O/bench_shard.log" 2>&1 || { tail -20 "$O/bench_shard.log"; exit 1; }
show "$O/bench_shard.log" shard
cd /tmp && export TMPDIR=/tmp
step kt3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt3" -o kt3 -- python "$R/bench.py" --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt3.log" 2>&1 || { tail -20 "$O/bench_kt3.log"; exit 1; }
step pmc3
P3="--steps 5 --warmup 1 --no-cpu-baseline --oracle-stride 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf3" -o pmcf3 -- python "$R/bench.py" $P3 > "$O/bench_pmcf3.log" 2>&1 || { tail -20 "$O/bench_pmcf3.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmcw3" -o pmcw3 -- python "$R/bench.py" $P3 > "$O/bench_pmcw3.log" 2>&1 || { tail -20 "$O/bench_pmcw3.log"; exit 1; }
step done
