#!/bin/bash
# round 5: kernel 11 row-stream depth (NB 8 / 10 / 12 iterations in flight, 8-B tile records) at config 2,
# interleaved on one box (scratch libraries librfx_k11nb*.so, RFX_LIB); the merge and rehearsal suites
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05h; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"))'
for i in 1 2; do for nb in 8 12; do
RFX_ALLOW_STALE_LIB=1 RFX_LIB=$R/rag-foundation_amd/rfx/librfx_k11nb$nb.so timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2_nb${nb}_$i.log 2>&1 || { tail -30 $O/bench_cfg2_nb${nb}_$i.log; exit 1; }
echo -n "nb$nb "; python3 -c "$S" < $O/bench_cfg2_nb${nb}_$i.log
done; done
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2_prod.log 2>&1 || { tail -30 $O/bench_cfg2_prod.log; exit 1; }
echo -n "prod "; python3 -c "$S" < $O/bench_cfg2_prod.log
RFX_ALLOW_STALE_LIB=1 RFX_LIB=$R/rag-foundation_amd/rfx/librfx_k11nb12.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_screen_valu.py > $O/pytest_k11_nb12.log 2>&1 || { tail -30 $O/pytest_k11_nb12.log; exit 1; }
tail -1 $O/pytest_k11_nb12.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_merge.py tests/test_gpu_bench_rehearsal.py > $O/pytest_merge_rehearsal.log 2>&1 || { tail -40 $O/pytest_merge_rehearsal.log; exit 1; }
tail -1 $O/pytest_merge_rehearsal.log
