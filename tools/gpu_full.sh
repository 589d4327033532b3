#!/bin/bash
# Full evidence session: smoke -> GPU parity tests -> default bench -> scan ablations ->
# rocprofv3 kernel-trace stats of the bench -> two separate PMC passes (FETCH_SIZE, WRITE_SIZE).
# Every GPU step has its own time limit; the chain stops at the first failure (no retries).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p "$O"
export PYTHONDONTWRITEBYTECODE=1
BENCH_ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3"}
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed rc=$?"; tail -30 "$O/smoke.log"; exit 1; }
echo "smoke ok"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > "$O/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -60 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
timeout -k 10 400 python bench.py $BENCH_ARGS > "$O/bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -30 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
if [ -n "$VARIANTS" ]; then
  timeout -k 10 300 python tools/scan_variants.py $VARIANTS > "$O/variants.json" 2> "$O/variants.err" || { echo "variants rc=$?"; tail -20 "$O/variants.err"; exit 1; }
  cat "$O/variants.json"
fi
[ -n "$SKIP_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
rm -rf "$O/prof_kt" "$O/prof_fetch" "$O/prof_write"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_kt" -o kt -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_kt.log" 2>&1 || { echo "kt rc=$?"; tail -20 "$O/bench_kt.log"; exit 1; }
tail -1 "$O/bench_kt.log"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/prof_fetch" -o pmc -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_fetch.log" 2>&1 || { echo "fetch pmc rc=$?"; tail -20 "$O/bench_fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/prof_write" -o pmc -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_write.log" 2>&1 || { echo "write pmc rc=$?"; tail -20 "$O/bench_write.log"; exit 1; }
find "$O/prof_kt" "$O/prof_fetch" "$O/prof_write" -type f
