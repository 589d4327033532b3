#!/bin/bash
# Round 6, first GPU call: VMM probe, smoke, the tests of this round's changes, then the nq benches.
set -o pipefail
O=gpurun_out/r06a
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 120 tools/r06/vmm_probe > "$O/vmm_probe.log" 2>&1; echo "vmm_probe rc=$?"; cat "$O/vmm_probe.log"
tools/r06/gpu_tests.sh "$O" tests/test_gpu_screen_w2.py tests/test_gpu_screen.py tests/test_gpu_merge.py tests/test_gpu_sharded.py tests/test_dist_gpu.py tests/test_gpu_union.py || exit 1
tools/r06/gpu_bench_nq.sh "$O"
