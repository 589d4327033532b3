#!/bin/bash
# Round 6: the select with the in-launch fallback (RFX_SELECT_FB=1) against the three launches (=0),
# interleaved: the 8-GPU shard step and config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06b}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"))'
for i in 1 2; do
  for v in 1 0; do
    RFX_SELECT_FB=$v timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/shard_fb${v}_$i.log 2>&1 || { tail -20 $O/shard_fb${v}_$i.log; exit 1; }
    echo -n "shard fb=$v $i: "; python3 -c "$S" < $O/shard_fb${v}_$i.log
    RFX_SELECT_FB=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/cfg3_fb${v}_$i.log 2>&1 || { tail -20 $O/cfg3_fb${v}_$i.log; exit 1; }
    echo -n "cfg3 fb=$v $i: "; python3 -c "$S" < $O/cfg3_fb${v}_$i.log
  done
done
