#!/bin/bash
# Round 6: kernel 11's list path seeded by one selection over the first two kept chunks, against the
# previous build (librfx_base.so): kernel 11's tests, then 300k / 1M x 768 f32 at nq 1 and 8, and config 2,
# interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06hy}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"))'
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_screen_valu.py tests/test_gpu_screen.py tests/test_gpu_sharded.py tests/test_gpu_filters.py tests/test_gpu_union.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -1 $O/pytest_k11.log
for cfg in "300000 1" "300000 8" "1000000 1" "1000000 8" "100000 1"; do
  set -- $cfg
  for v in new base; do
    if [ $v = base ]; then export RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1; else unset RFX_LIB RFX_ALLOW_STALE_LIB; fi
    timeout -k 10 300 python -u bench.py --rows $1 --dtype f32 --nq $2 --steps 500 --warmup 50 --event-stride 16 --no-cpu-baseline > $O/r$1_nq$2_$v.log 2>&1 || { tail -20 $O/r$1_nq$2_$v.log; exit 1; }
    echo -n "rows=$1 nq=$2 $v: "; python3 -c "$S" < $O/r$1_nq$2_$v.log
  done
done
