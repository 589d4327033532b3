#!/bin/bash
# One GPU session: smoke -> parity tests -> short bench.  Every GPU step has its own time limit and
# the chain stops at the first failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
TESTS=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 ${TEST_TIMEOUT:-700} python -m pytest $TESTS -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest.log; exit 1; }
tail -3 gpurun_out/pytest.log
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
