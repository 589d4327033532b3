#!/bin/bash
# round 3: kernel 10's slot-table refresh at every one of the first 16 tiles (MODE 16) against the
# production schedule: slow-path entries and time at config 3 (10M) and the 8-GPU shard (1.25M)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03aa; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --variants 8032,8048,8000,8016 --rounds 6 > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 8032,8048,8000,8016 --rounds 8 --burst 100 > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -h "slow_path\|min" $O/k10_10m.txt $O/k10_shard.txt
