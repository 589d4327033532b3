#!/bin/bash
# round 5: kernel 10's sorted-merge fold (debug MODE 16384: a wave with >= 8 passes in some lane folds by
# one bitonic merge instead of pop-loop trips) against production, shard and 10M, on one box
# (scratch debug library librfx_dbg_sm.so built from the worktree with the mode)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05i; mkdir -p $O
export RFX_ALLOW_STALE_LIB=1 RFX_LIB=$R/rag-foundation_amd/rfx/librfx_dbg_sm.so
V=102097152,102113536,102097664
timeout -k 10 500 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_shard.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
grep '"variant"' $O/k10_shard.txt
timeout -k 10 500 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_10m.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
grep '"variant"' $O/k10_10m.txt
timeout -k 10 300 python -u tools/k10_trips.py --variant 102121728 > $O/k10_trips_sm.json 2>&1 || { tail -20 $O/k10_trips_sm.json; exit 1; }
grep -h "total" $O/k10_trips_sm.json
