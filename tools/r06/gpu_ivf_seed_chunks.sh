#!/bin/bash
# Round 6: the IVF list scan's seeded chunks per wave, 2 (production) against 3 and 4 (librfx_s3.so,
# librfx_s4.so built with kSeedChunks 3 / 4), config 5 (tools/bench_ivf.py) interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06ivf2}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_batch"], d.get("achieved_list_GBps"), d.get("recall_at_k"))'
for i in 1 2; do
  timeout -k 10 600 python -u tools/bench_ivf.py > $O/ivf_s2_$i.log 2>&1 || { tail -20 $O/ivf_s2_$i.log; exit 1; }
  echo -n "s2 $i: "; python3 -c "$S" < $O/ivf_s2_$i.log
  for n in 3 4; do
    RFX_LIB=$R/rag-foundation_amd/rfx/librfx_s$n.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 600 python -u tools/bench_ivf.py > $O/ivf_s${n}_$i.log 2>&1 || { tail -20 $O/ivf_s${n}_$i.log; exit 1; }
    echo -n "s$n $i: "; python3 -c "$S" < $O/ivf_s${n}_$i.log
  done
done
