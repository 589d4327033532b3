#!/bin/bash
# round 5, first session: baseline on this box (config 3 default step, the 8-GPU shard step), kernel 10
# epilogue-placement / partner-bound variants at the shard and at 10M (validated against production),
# slow-path trips per tile for production and the late epilogue, and the PMC counter list of gfx950
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("phases_ms"), d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check",{}).get("ok"), d["build_id"])'
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list failed"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
V=80000000,80131072,80262144,80393216,80524288,80655360,80917504
timeout -k 10 400 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -v amdgpu $O/k10_shard.txt | tail -40
timeout -k 10 400 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --variants $V > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
grep -v amdgpu $O/k10_10m.txt | tail -30
timeout -k 10 300 python -u tools/k10_trips.py > $O/k10_trips_prod.json 2>&1 || { tail -20 $O/k10_trips_prod.json; exit 1; }
timeout -k 10 300 python -u tools/k10_trips.py --variant 80139264 > $O/k10_trips_late.json 2>&1 || { tail -20 $O/k10_trips_late.json; exit 1; }
grep -h "total" $O/k10_trips_*.json
# the round-5 correctness changes: one score rule for the exact plans, the row-offset re-score, the widened e2,
# dropped copies as a store state, union builds off the global lock
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_screen_capacity.py tests/test_gpu_union.py tests/test_gpu_sharded.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_screen_valu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
