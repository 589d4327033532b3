#!/bin/bash
# Round 6: where kernel 11's time goes with several questions (100k x 768 f32, nq 8 and 2): timing-only
# ablations (RFX_K11_ABLATE: 2 no row stream, 8 no last-block work, 16 no re-score + rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06n8a}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'
for nq in 8 2; do for a in 0 2 8 16 10; do
  RFX_K11_ABLATE=$a timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq $nq --steps 1000 --warmup 100 --event-stride 16 --no-cpu-baseline --oracle-stride 0 > $O/nq${nq}_a$a.log 2>&1 || { tail -20 $O/nq${nq}_a$a.log; exit 1; }
  echo -n "nq=$nq ablate=$a: "; python3 -c "$S" < $O/nq${nq}_a$a.log
done; done
