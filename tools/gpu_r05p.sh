#!/bin/bash
# round 5: kernel 11 touching the record heads' exact rows into the cache before its bound / survivors
# (LDS-DMA into a sink) — config 2 interleaved against the previous build (scratch librfx_e805.so), the
# kernel-11 tests, and its phases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05p; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d.get("oracle_check", {}).get("ok"), d.get("build_id"))'
C2="--rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline"
for i in 1 2; do
timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2_new_$i.log 2>&1 || { tail -30 $O/bench_cfg2_new_$i.log; exit 1; }
echo -n "new "; python3 -c "$S" < $O/bench_cfg2_new_$i.log
RFX_ALLOW_STALE_LIB=1 RFX_LIB=$R/rag-foundation_amd/rfx/librfx_e805.so timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2_old_$i.log 2>&1 || { tail -30 $O/bench_cfg2_old_$i.log; exit 1; }
echo -n "old "; python3 -c "$S" < $O/bench_cfg2_old_$i.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_screen_valu.py > $O/pytest_k11.log 2>&1 || { tail -30 $O/pytest_k11.log; exit 1; }
tail -1 $O/pytest_k11.log
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
grep -v amdgpu $O/k11_phases.json | head -30
