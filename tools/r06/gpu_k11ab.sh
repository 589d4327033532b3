#!/bin/bash
# Round 6: kernel 11 with the last block's own entries re-scored alongside its record loads, against the
# library before it (rfx/ab/librfx_k11old.so); config 2 interleaved on one box, then the kernel-11 tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/${1:-gpurun_out/r06e}; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"))'
C2="--rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2_new_$i.log 2>&1 || { tail -30 $O/bench_cfg2_new_$i.log; exit 1; }
  echo -n "new $i: "; python3 -c "$S" < $O/bench_cfg2_new_$i.log
  RFX_LIB=$R/rag-foundation_amd/rfx/ab/librfx_k11old.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2_old_$i.log 2>&1 || { tail -30 $O/bench_cfg2_old_$i.log; exit 1; }
  echo -n "old $i: "; python3 -c "$S" < $O/bench_cfg2_old_$i.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_screen_valu.py tests/test_gpu_fused.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -1 $O/pytest_k11.log
