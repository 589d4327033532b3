#!/bin/bash
# Round 6: config 4 (one GPU's shard, 12.5M x 1024 f16) and config 5 (IVF-Flat int8 per-GPU shard) on the
# current build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06c45}; mkdir -p $O
timeout -k 10 500 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg4_shard.log 2>&1 || { tail -20 $O/bench_cfg4_shard.log; exit 1; }
tail -1 $O/bench_cfg4_shard.log | cut -c1-300
timeout -k 10 600 python -u tools/bench_ivf.py > $O/ivf_bench.log 2>&1 || { tail -20 $O/ivf_bench.log; exit 1; }
tail -1 $O/ivf_bench.log | cut -c1-400
