#!/bin/bash
# Round 6: two-pass (2-wave kernel 10) against the exact scan at the micro-batcher's batch sizes.
# Usage: tools/r06/gpu_bench_nq.sh OUTDIR
set -o pipefail
O=${1:-gpurun_out/r06}
mkdir -p "$O"
export TMPDIR=/tmp
for nq in 16 32 64; do
  for scan in auto exact; do
    timeout -k 10 300 python -u bench.py --nq $nq --scan $scan --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_10m_nq${nq}_${scan}.log" 2>&1 || { echo "bench nq=$nq $scan rc=$?"; tail -20 "$O/bench_10m_nq${nq}_${scan}.log"; exit 1; }
    tail -1 "$O/bench_10m_nq${nq}_${scan}.log" | cut -c1-300
  done
done
for nq in 16 32 64; do
  for scan in auto exact; do
    timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq $nq --scan $scan --steps 200 --warmup 20 --no-cpu-baseline > "$O/bench_100k_f32_nq${nq}_${scan}.log" 2>&1 || { echo "bench f32 nq=$nq $scan rc=$?"; tail -20 "$O/bench_100k_f32_nq${nq}_${scan}.log"; exit 1; }
    tail -1 "$O/bench_100k_f32_nq${nq}_${scan}.log" | cut -c1-300
  done
done
