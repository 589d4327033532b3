#!/bin/bash
# Round 6: the 2-wave kernel 10's workgroup count on a small store (100k x 768 f32, the config-2 store) and on
# 10M rows, batches of 32 questions (RFX_SCREEN_W2_BLOCKS overrides plan_scan_screen's count).
set -o pipefail
O=${1:-gpurun_out/r06t}
mkdir -p "$O"
export TMPDIR=/tmp
for b in 64 128 192 256 384; do
  RFX_SCREEN_W2_BLOCKS=$b timeout -k 10 200 python -u bench.py --rows 100000 --dtype f32 --nq 32 --steps 300 --warmup 30 --no-cpu-baseline > "$O/w2_100k_b$b.log" 2>&1 || { echo "b=$b rc=$?"; exit 1; }
  echo "100k f32 nq32 blocks=$b: $(tail -1 "$O/w2_100k_b$b.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
for b in 256 512; do
  RFX_SCREEN_W2_BLOCKS=$b timeout -k 10 200 python -u bench.py --nq 32 --steps 20 --warmup 3 --no-cpu-baseline > "$O/w2_10m_b$b.log" 2>&1 || { echo "b=$b rc=$?"; exit 1; }
  echo "10M bf16 nq32 blocks=$b: $(tail -1 "$O/w2_10m_b$b.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["frac"])')"
done
