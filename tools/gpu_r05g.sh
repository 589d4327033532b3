#!/bin/bash
# round 5: kernel 10's integer pass threshold in the slow path (production) against the float test, on the
# per-tile-barrier schedule; config 3 and the 8-GPU shard step on one box (interleaved); config 2 with the
# lazy kernel-11 launch order; then the GPU suites of the paths touched
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05g; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"), d.get("phases_ms"))'
V=102097152,106291456,80000000,102097664
timeout -k 10 500 python -u tools/k10_variants.py --rows 1250000 --rounds 6 --burst 50 --validate --variants $V > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_shard.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 500 python -u tools/k10_variants.py --rows 10000000 --rounds 4 --burst 20 --validate --variants $V > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
grep -A1 "\"[0-9]*\": {" $O/k10_10m.txt | grep -v "^--" | paste - - | awk '{print $1, $3}'
timeout -k 10 300 python -u tools/k10_trips.py --variant 102105344 > $O/k10_trips_int.json 2>&1 || { tail -20 $O/k10_trips_int.json; exit 1; }
grep -h "total" $O/k10_trips_int.json
for i in 1 2; do
timeout -k 10 300 python -u bench.py > $O/bench_cfg3_$i.log 2>&1 || { tail -30 $O/bench_cfg3_$i.log; exit 1; }
python3 -c "$S" < $O/bench_cfg3_$i.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc_$i.log 2>&1 || { tail -30 $O/bench_shard_fc_$i.log; exit 1; }
python3 -c "$S" < $O/bench_shard_fc_$i.log
done
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
python3 -c "$S" < $O/bench_cfg2.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_screen_valu.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py tests/test_gpu_screen.py tests/test_gpu_fused.py tests/test_gpu_screen_capacity.py tests/test_gpu_union.py tests/test_gpu_filters.py tests/test_gpu_merge.py tests/test_gpu_bench_rehearsal.py > $O/pytest_paths.log 2>&1 || { tail -40 $O/pytest_paths.log; exit 1; }
tail -3 $O/pytest_paths.log
