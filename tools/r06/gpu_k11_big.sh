#!/bin/bash
# Round 6: kernel 11 on larger stores (list path: > 128 rows per wave), nq 1 and 8, with and without the
# waves' list offers (RFX_K11_ABLATE=64, timing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06big}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"].get("scan_kernel","")[:30])'
for rows in 300000 1000000; do for nq in 1 8; do for a in 0 64; do
  RFX_K11_ABLATE=$a timeout -k 10 300 python -u bench.py --rows $rows --dtype f32 --nq $nq --steps 500 --warmup 50 --event-stride 16 --no-cpu-baseline --oracle-stride 0 > $O/r${rows}_nq${nq}_a$a.log 2>&1 || { tail -20 $O/r${rows}_nq${nq}_a$a.log; exit 1; }
  echo -n "rows=$rows nq=$nq ablate=$a: "; python3 -c "$S" < $O/r${rows}_nq${nq}_a$a.log
done; done; done
