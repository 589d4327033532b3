#!/bin/bash
# round 3: kernel 10 at the 8-GPU shard size (1.25M rows): slow-path entries (MODE 32 count), production,
# slow path never taken (512), no fold (1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 8032,8000,8512,8001 --rounds 6 --burst 100 > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
cat $O/k10_shard.txt
