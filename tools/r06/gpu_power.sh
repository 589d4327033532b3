#!/bin/bash
# Round 6 (first step): package power and sclk (rocm-smi) during 16-s bursts of kernel 10
# variants on config 3 (10M x 768, nq 256), and the in-kernel clock of production from per-block
# s_memtime / s_memrealtime stamps (debug MODE 65536).  Variants (10^8 RING + MODE): production 1010485760,
# no fold 1010485761, no fold + no corpus stream 1010485769; the 64-queries-per-wave kernel: 64, its
# no-fold 65 and no-fold-no-stream 73.
set -o pipefail
O=${1:-gpurun_out/r06p}
mkdir -p "$O"
export TMPDIR=/tmp
# the 64-queries-per-wave kernel's answers first (every two-pass test, on it)
RFX_K10_Q64=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen.py \
  tests/test_gpu_screen_capacity.py > "$O/pytest_q64.log" 2>&1 || { echo "q64 tests rc=$?"; tail -30 "$O/pytest_q64.log"; exit 1; }
tail -1 "$O/pytest_q64.log"
sample() {  # $1 = output file: rocm-smi every ~0.5 s while the burst runs
  for i in $(seq 1 12); do
    rocm-smi -c -P >> "$1" 2>&1
    sleep 0.5
  done
}
for v in 1010485760 1010485761 1010485769 64 65 73; do
  [ "$v" -lt 100 ] && export RFX_K10_Q64=1 || unset RFX_K10_Q64
  timeout -k 10 200 python -u tools/k10_variants.py --variants $v --seconds 16 --rounds 1 --burst 5 > "$O/run_$v.json" 2> "$O/run_$v.err" &
  pid=$!
  for i in $(seq 1 240); do grep -q "burst start" "$O/run_$v.err" 2>/dev/null && break; sleep 0.5; done
  sleep 2  # (past the burst's first launches)
  sample "$O/smi_$v.txt"
  wait $pid || { echo "variant $v rc=$?"; tail -5 "$O/run_$v.err"; exit 1; }
  tail -2 "$O/run_$v.json"
done
unset RFX_K10_Q64
timeout -k 10 300 python -u tools/k10_block_times.py --reps 10 > "$O/block_clocks_prod.json" 2> "$O/block_clocks.err" || { echo "clocks rc=$?"; tail -5 "$O/block_clocks.err"; exit 1; }
grep -E "clock_mhz_med|dur_med_ns|end_max_ns\"" "$O/block_clocks_prod.json" | head -5
