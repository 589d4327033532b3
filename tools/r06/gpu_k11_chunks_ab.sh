#!/bin/bash
# Round 6: kernel 11 kept-score chunks, 2 (librfx_base.so, 250 workgroups) against 4 (this build) at 250 /
# 192 / 160 workgroups, config 2, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06kc}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"))'
C2="--rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline"
for i in 1 2 3; do
  RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u bench.py $C2 > $O/cfg2_c2_b250_$i.log 2>&1 || { tail -20 $O/cfg2_c2_b250_$i.log; exit 1; }
  echo -n "chunks=2 blocks=250 $i: "; python3 -c "$S" < $O/cfg2_c2_b250_$i.log
  for nb in 250 192 160; do
    RFX_VALU_BLOCKS=$nb timeout -k 10 300 python -u bench.py $C2 > $O/cfg2_c4_b${nb}_$i.log 2>&1 || { tail -20 $O/cfg2_c4_b${nb}_$i.log; exit 1; }
    echo -n "chunks=4 blocks=$nb $i: "; python3 -c "$S" < $O/cfg2_c4_b${nb}_$i.log
  done
done
