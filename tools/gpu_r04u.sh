#!/bin/bash
# round 4: kernel 10's block tail (debug MODE 65536 per-block wall clocks) at the 8-GPU shard and 10M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 240 python -u tools/k10_block_times.py --rows 1250000 > $O/k10_block_times_shard.json 2>&1 || { tail -20 $O/k10_block_times_shard.json; exit 1; }
grep -v amdgpu $O/k10_block_times_shard.json | tr -d ' \n'; echo
timeout -k 10 300 python -u tools/k10_block_times.py --rows 10000000 --reps 10 > $O/k10_block_times_10m.json 2>&1 || { tail -20 $O/k10_block_times_10m.json; exit 1; }
grep -v amdgpu $O/k10_block_times_10m.json | tr -d ' \n'; echo
