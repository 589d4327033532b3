#!/bin/bash
# round 3: kernel-10 breakdown (debug library): production, no fold, no stream, neither; slow-path count
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --variants 832,800,801,808,809,400,600 --rounds 4 > $O/variants.json 2> $O/variants.err || { tail -5 $O/variants.err; exit 1; }
cat $O/variants.json
