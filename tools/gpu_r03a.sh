#!/bin/bash
# round 3: first run of the two-pass scan (kernel 10) parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_screen.py > gpurun_out/r03a_screen.log 2>&1
rc=$?
tail -30 gpurun_out/r03a_screen.log
exit $rc
