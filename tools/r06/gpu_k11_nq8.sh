#!/bin/bash
# Round 6: kernel 11 with several questions (100k x 768 f32, nq 2 / 4 / 8): time, and the no-offer ablation
# (RFX_K11_ABLATE=64, timing only) — what the waves' list inserts cost there.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06n8}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"].get("scan_kernel","")[:40])'
for nq in 2 4 8; do for a in 0 64; do
  RFX_K11_ABLATE=$a timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq $nq --steps 1000 --warmup 100 --event-stride 16 --no-cpu-baseline --oracle-stride 0 > $O/nq${nq}_a$a.log 2>&1 || { tail -20 $O/nq${nq}_a$a.log; exit 1; }
  echo -n "nq=$nq ablate=$a: "; python3 -c "$S" < $O/nq${nq}_a$a.log
done; done
