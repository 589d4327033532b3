#!/bin/bash
# round 5: kernel 11, the last block's bound by one key per thread (counting) against build 832adb65 (k-round extraction)
# config 2 interleaved on one box; the last block's phases; the
# GPU suites of the kernel-11 paths
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05v; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"))'
C2="--rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_screen_valu.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -2 $O/pytest_k11.log
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2_new_$i.log 2>&1 || { tail -30 $O/bench_cfg2_new_$i.log; exit 1; }
echo -n "new $i: "; python3 -c "$S" < $O/bench_cfg2_new_$i.log
RFX_LIB=$R/rag-foundation_amd/rfx/ab/librfx_832a.so RFX_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2_old_$i.log 2>&1 || { tail -30 $O/bench_cfg2_old_$i.log; exit 1; }
echo -n "old $i: "; python3 -c "$S" < $O/bench_cfg2_old_$i.log
done
timeout -k 10 300 python -u tools/k11_phases.py --reps 160 > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
grep -v amdgpu $O/k11_phases.json | tr -d '\n '; echo
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_merge.py tests/test_gpu_sharded.py tests/test_gpu_union.py tests/test_gpu_filters.py tests/test_gpu_fused.py tests/test_gpu_bench_rehearsal.py > $O/pytest_paths.log 2>&1 || { tail -40 $O/pytest_paths.log; exit 1; }
tail -2 $O/pytest_paths.log
