#!/bin/bash
# Round 6: GPU tests on one box.  Usage: tools/r06/gpu_tests.sh OUTDIR [pytest targets...]
set -o pipefail
O=${1:-gpurun_out/r06}; shift
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$O/smoke.log"; exit 1; }
timeout -k 10 1500 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu "$@" > "$O/pytest.log" 2>&1
rc=$?
tail -5 "$O/pytest.log"
exit $rc
