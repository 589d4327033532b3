#!/bin/bash
# Round 6: do the virtual-memory mappings (4-KB granularity, rows and int8 copy mapped with hipMemMap) cost
# TLB reach?  Store memory from hipMemCreate + hipMemMap (default) against hipMalloc (RFX_VMM=0), interleaved
# on one box: config 2, the 8-GPU shard, config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06v}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"))'
for i in 1 2; do
  for v in 1 0; do
    RFX_VMM=$v timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/cfg2_vmm${v}_$i.log 2>&1 || { tail -20 $O/cfg2_vmm${v}_$i.log; exit 1; }
    echo -n "cfg2 vmm=$v $i: "; python3 -c "$S" < $O/cfg2_vmm${v}_$i.log
    RFX_VMM=$v timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/shard_vmm${v}_$i.log 2>&1 || { tail -20 $O/shard_vmm${v}_$i.log; exit 1; }
    echo -n "shard vmm=$v $i: "; python3 -c "$S" < $O/shard_vmm${v}_$i.log
    RFX_VMM=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/cfg3_vmm${v}_$i.log 2>&1 || { tail -20 $O/cfg3_vmm${v}_$i.log; exit 1; }
    echo -n "cfg3 vmm=$v $i: "; python3 -c "$S" < $O/cfg3_vmm${v}_$i.log
  done
done
