#!/bin/bash
# round 5: kernel 10 slow-path variants on production (per-tile barrier + publish-on-change), scratch
# debug library librfx_dbg_x.so: two passing values per pop-loop trip (16777216), the integer pass
# mask by a shift-or tree (33554432), both, and s_setprio in the slow path (2048)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp RFX_ALLOW_STALE_LIB=1 RFX_LIB=$GRAFT_REPO_ROOT/rag-foundation_amd/rfx/librfx_dbg_x.so
O=$GRAFT_REPO_ROOT/gpurun_out/r05o; mkdir -p $O
V=1010485760,1027262976,1044040192,1060817408,1010487808
timeout -k 10 600 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_x_shard.txt 2>&1 || { tail -20 $O/k10_x_shard.txt; exit 1; }
grep '"variant"' $O/k10_x_shard.txt
timeout -k 10 600 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_x_10m.txt 2>&1 || { tail -20 $O/k10_x_10m.txt; exit 1; }
grep '"variant"' $O/k10_x_10m.txt
