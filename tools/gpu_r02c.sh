#!/bin/bash
# Round-2 GPU session C: smoke, the whole -m gpu suite, the default bench (oracle check + CPU
# baseline), rocprofv3 kernel stats of the bench and FETCH_SIZE / WRITE_SIZE passes for the
# traffic summary.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02c"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=8 -v --timeout 420 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
fi
step bench
timeout -k 10 400 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --no-cpu-baseline --oracle-stride 0"
step kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $B --steps 20 --warmup 5 > "$O/bench_kt.log" 2>&1 || { tail -20 "$O/bench_kt.log"; exit 1; }
step fetch
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf" -o pmcf -- $B --steps 4 --warmup 1 > "$O/bench_pmcf.log" 2>&1 || { tail -20 "$O/bench_pmcf.log"; exit 1; }
step write
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmcw" -o pmcw -- $B --steps 4 --warmup 1 > "$O/bench_pmcw.log" 2>&1 || { tail -20 "$O/bench_pmcw.log"; exit 1; }
step done
cd "$R" || exit 1
if [ -n "$CFG2" ]; then
step cfg2
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --steps 3000 --warmup 200"
timeout -k 10 300 python -u bench.py $C2 > "$O/bench_cfg2.log" 2>&1 || { tail -20 "$O/bench_cfg2.log"; exit 1; }
tail -1 "$O/bench_cfg2.log" | cut -c1-300
timeout -k 10 300 python -u bench.py $C2 --unfused --no-cpu-baseline > "$O/bench_cfg2_unfused.log" 2>&1 || { tail -20 "$O/bench_cfg2_unfused.log"; exit 1; }
tail -1 "$O/bench_cfg2_unfused.log" | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt2 -- python "$R/bench.py" $C2 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt2.log" 2>&1 || { tail -20 "$O/bench_kt2.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf2" -o pmcf2 -- python "$R/bench.py" --rows 100000 --dim 768 --dtype f32 --nq 1 --steps 50 --warmup 10 --no-cpu-baseline --oracle-stride 0 > "$O/bench_pmcf2.log" 2>&1 || { tail -20 "$O/bench_pmcf2.log"; exit 1; }
step cfg2done
fi
