#!/bin/bash
# round 5: the sharded search's Python path against the one-call C path; kernel 10 with one wait + barrier
# per tile (debug TB) on round 4's fold; kernel 11's exact fallback back inside its launch (claimed
# virtual blocks, per-device launch order): its tests, config 2 and its rocprof summary
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["metric"][:12], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])'
timeout -k 10 300 python -u tools/debug_sharded_paths.py > $O/debug_sharded_paths.log 2>&1 || { tail -30 $O/debug_sharded_paths.log; }
grep -v amdgpu $O/debug_sharded_paths.log | head -40
V=80000000,122097152,102097152,122621440,122097664,122097153
timeout -k 10 500 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_shard.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 500 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_10m.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 300 python -u tools/k10_trips.py --variant 122105344 > $O/k10_trips_tb.json 2>&1 || { tail -20 $O/k10_trips_tb.json; exit 1; }
timeout -k 10 300 python -u tools/k10_trips.py --variant 80008192 > $O/k10_trips_prod.json 2>&1 || { tail -20 $O/k10_trips_prod.json; exit 1; }
grep -h "total" $O/k10_trips_*.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_screen_valu.py tests/test_gpu_fused.py > $O/pytest_k11.log 2>&1 || { tail -40 $O/pytest_k11.log; exit 1; }
tail -3 $O/pytest_k11.log
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
python3 -c "$S" < $O/bench_cfg2.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_cfg2 -o cfg2 -- python3 $GRAFT_REPO_ROOT/bench.py --rows 100000 --dtype f32 --nq 1 --steps 400 --warmup 50 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_cfg2.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_cfg2.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof_cfg2 -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-200
