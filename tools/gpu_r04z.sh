#!/bin/bash
# round 4: is kernel 11's row stream latency-bound per wave?  Its phases with fewer, longer waves
# (RFX_VALU_BLOCKS 128 / 192 against the default 256 blocks of 4 waves)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
for b in 256 192 128; do
  RFX_VALU_BLOCKS=$b timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases_b$b.json 2>&1 || { tail -20 $O/k11_phases_b$b.json; exit 1; }
  echo "blocks $b"; grep -v amdgpu $O/k11_phases_b$b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['blocks'], d['median'])"
done
