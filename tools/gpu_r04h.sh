#!/bin/bash
# round 4: kernel 10's deferred slow path (MODE 16384: list inserts under the next tile's MFMAs), with and
# without slow-path priority (2048), at the 8-GPU shard and at 10M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 800000,816384,818432,816416,800032 --rounds 8 --burst 100 > $O/k10_shard_defer.txt 2>&1 || { tail -20 $O/k10_shard_defer.txt; exit 1; }
grep -h "slow_path\|min\|\"8" $O/k10_shard_defer.txt
timeout -k 10 300 python -u tools/k10_variants.py --variants 800000,816384,818432 --rounds 6 > $O/k10_10m_defer.txt 2>&1 || { tail -20 $O/k10_10m_defer.txt; exit 1; }
grep -h "min\|\"8" $O/k10_10m_defer.txt
