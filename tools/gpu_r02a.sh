#!/bin/bash
# Round-2 GPU session A: smoke, full-size parity (cfg3 10M rows, cfg4 12.5M-row shard), bench with
# its oracle check, rocprofv3 kernel stats + clock (GRBM_GUI_ACTIVE) of the bench, cfg4-shard bench
# with kernel stats and FETCH_SIZE.  Every GPU step has its own time limit; the first failure ends
# the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02a"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
step() { echo "== $1 $(date +%T)"; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
step fullsize
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 420 --timeout-method thread > "$O/fullsize.log" 2>&1 || { tail -40 "$O/fullsize.log"; exit 1; }
tail -3 "$O/fullsize.log"
step bench
timeout -k 10 400 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
cd /tmp && export TMPDIR=/tmp
step kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --oracle-stride 0 > "$O/bench_kt.log" 2>&1 || { tail -20 "$O/bench_kt.log"; exit 1; }
step clk
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$O/clk" -o clk -- python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --oracle-stride 0 > "$O/bench_clk.log" 2>&1 || { tail -20 "$O/bench_clk.log"; exit 1; }
python "$R/tools/clock_summary.py" "$O/clk" > "$O/clock.txt" 2>&1; tail -5 "$O/clock.txt"
step cfg4
C4="--rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline"
timeout -k 10 400 python -u "$R/bench.py" $C4 > "$O/bench_cfg4.log" 2>&1 || { tail -20 "$O/bench_cfg4.log"; exit 1; }
tail -1 "$O/bench_cfg4.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt4" -o kt4 -- python "$R/bench.py" $C4 --steps 10 --warmup 2 --oracle-stride 0 > "$O/bench_kt4.log" 2>&1 || { tail -20 "$O/bench_kt4.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc4" -o pmc4 -- python "$R/bench.py" $C4 --steps 4 --warmup 1 --oracle-stride 0 > "$O/bench_pmc4.log" 2>&1 || { tail -20 "$O/bench_pmc4.log"; exit 1; }
step done
