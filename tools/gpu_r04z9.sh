#!/bin/bash
# round 4: kernel 11 runs its exact fallback inside its own launch for a lone question (no gated launch
# behind it): kernel 11 / sharded / union / boundary tests (forced and natural fallbacks, one-block
# stores), config 2 and its phases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z9; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d["phases_ms"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_screen_valu.py tests/test_gpu_sharded.py tests/test_gpu_union.py tests/test_gpu_boundary.py tests/test_gpu_screen_capacity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
tail -1 $O/bench_cfg2.log | python3 -c "$S"
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
grep -v amdgpu $O/k11_phases.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['median'])"
