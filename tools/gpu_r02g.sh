#!/bin/bash
# Round-2 GPU session G: the -m gpu suite (kernel 8 as the d-1024 kernel, the LDS-staged fused
# merge of the one-launch VALU search), config 2 with its kernel stats, and the config-4 shard
# bench through kernel 8.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-r02g}"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=8 -q --timeout 420 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
fi
step cfg2
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 300"
timeout -k 10 300 python -u bench.py $C2 --event-stride 16 > "$O/bench_cfg2.log" 2>&1 || { tail -20 "$O/bench_cfg2.log"; exit 1; }
tail -1 "$O/bench_cfg2.log" | cut -c1-200
step cfg4
timeout -k 10 300 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 20 --warmup 3 --oracle-stride 4 > "$O/bench_cfg4.log" 2>&1 || { tail -20 "$O/bench_cfg4.log"; exit 1; }
tail -1 "$O/bench_cfg4.log" | cut -c1-200
cd /tmp && export TMPDIR=/tmp
step kt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt2 -- python "$R/bench.py" $C2 --no-cpu-baseline --oracle-stride 0 --event-stride 16 > "$O/bench_kt2.log" 2>&1 || { tail -20 "$O/bench_kt2.log"; exit 1; }
step pmc2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf2" -o pmcf2 -- python "$R/bench.py" --rows 100000 --dim 768 --dtype f32 --nq 1 --steps 50 --warmup 10 --no-cpu-baseline --oracle-stride 0 > "$O/bench_pmcf2.log" 2>&1 || { tail -20 "$O/bench_pmcf2.log"; exit 1; }
step done
