#!/bin/bash
# Parity tests (optionally filtered) + scan timing variants + bench.  Stops at first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests/test_gpu_parity.py -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
timeout -k 10 300 python tools/scan_variants.py ${VARIANT_ARGS} > gpurun_out/variants.json 2> gpurun_out/variants.err || { echo "variants rc=$?"; tail -20 gpurun_out/variants.err; exit 1; }
cat gpurun_out/variants.json
timeout -k 10 400 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
