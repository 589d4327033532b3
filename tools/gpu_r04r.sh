#!/bin/bash
# round 4: how much of kernel 10's time is the pruning bound's warm-up?  RFX_DBG_KEEP_TAU=1 starts
# every launch from the previous launch's final slot table (no warm-up at all; debug library)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
for keep in 0 1; do
  if [ $keep = 1 ]; then export RFX_DBG_KEEP_TAU=1; fi
  timeout -k 10 240 python -u tools/k10_variants.py --rows 1250000 --variants 800000,800001 --rounds 8 --burst 100 > $O/k10_shard_keep$keep.txt 2>&1 || { tail -20 $O/k10_shard_keep$keep.txt; exit 1; }
  grep -v amdgpu $O/k10_shard_keep$keep.txt | tr -d ' \n'; echo
  timeout -k 10 300 python -u tools/k10_variants.py --rows 10000000 --variants 800000,800001 --rounds 4 --burst 30 > $O/k10_10m_keep$keep.txt 2>&1 || { tail -20 $O/k10_10m_keep$keep.txt; exit 1; }
  grep -v amdgpu $O/k10_10m_keep$keep.txt | tr -d ' \n'; echo
done
