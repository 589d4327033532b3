#!/bin/bash
# Round 6: what kernel 11's wave-list offers cost at config 2 (RFX_K11_ABLATE=64: no offers, timing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06o}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'
for i in 1 2; do for a in 0 64 2 8 72; do
  RFX_K11_ABLATE=$a timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline --oracle-stride 0 > $O/cfg2_ablate${a}_$i.log 2>&1 || { tail -20 $O/cfg2_ablate${a}_$i.log; exit 1; }
  echo -n "ablate=$a $i: "; python3 -c "$S" < $O/cfg2_ablate${a}_$i.log
done; done
