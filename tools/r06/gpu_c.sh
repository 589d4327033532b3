#!/bin/bash
# Round 6: the index tests on virtual-memory rows (address ranges never reused).
set -o pipefail
O=gpurun_out/r06c
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_filters.py tests/test_gpu_parity.py tests/test_gpu_union.py > "$O/vmm_fresh.log" 2>&1; echo "rc=$?"
grep -E "FAILED|ERROR" "$O/vmm_fresh.log" | head -20; tail -2 "$O/vmm_fresh.log"
