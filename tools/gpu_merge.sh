#!/bin/bash
# Merge changes check: full GPU suite, config-2 bench (split merge on / off), config-3 bench,
# config-2 kernel stats.  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
export PYTHONDONTWRITEBYTECODE=1
C2="--rows 100000 --dim 768 --nq 1 --dtype f32 --no-cpu-baseline"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_merge.log" 2>&1 || { echo "pytest failed rc=$?"; tail -60 "$O/pytest_merge.log"; exit 1; }
  tail -2 "$O/pytest_merge.log"
fi
timeout -k 10 200 python bench.py $C2 --steps 3000 --warmup 100 > "$O/bench_c2.log" 2>&1 || { echo "bench c2 rc=$?"; tail -30 "$O/bench_c2.log"; exit 1; }
tail -1 "$O/bench_c2.log"


timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_c3.log" 2>&1 || { echo "bench c3 rc=$?"; tail -30 "$O/bench_c3.log"; exit 1; }
tail -1 "$O/bench_c3.log"
cd /tmp && export TMPDIR=/tmp
rm -rf "$O/prof_c2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c2" -o kt -- python "$R/bench.py" $C2 --steps 1000 --warmup 50 > "$O/bench_c2_kt.log" 2>&1 || { echo "kt rc=$?"; tail -20 "$O/bench_c2_kt.log"; exit 1; }
head -6 "$O/prof_c2/kt_kernel_stats.csv"
timeout -k 10 200 python "$R/tools/merge_probe.py" > "$O/merge_probe.log" 2>&1 && cat "$O/merge_probe.log"
