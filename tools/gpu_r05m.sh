#!/bin/bash
# round 5: the whole -m gpu suite on the shipped build (as the driver runs it), then kernel 10's A/B of
# production (per-tile barrier + publish-on-change) against round 4's schedule on this box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=$GRAFT_REPO_ROOT/gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -60 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
V=1010485760,1002097152,800000000
timeout -k 10 500 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_prod_shard.txt 2>&1 || { tail -20 $O/k10_prod_shard.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_prod_shard.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 300 python -u tools/k10_trips.py > $O/k10_trips_prod.json 2>&1 || { tail -20 $O/k10_trips_prod.json; exit 1; }
grep -h "total" $O/k10_trips_prod.json
