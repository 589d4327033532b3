#!/bin/bash
# round 5: the per-tile-barrier kernel 10 and kernel 11's in-launch fallback (noinline claim loop) in
# production — config 3, the 8-GPU shard step (1-rank RCCL), config 2, config 4's shard; the in-process
# sharded search's host issue (RFX_DEVICES=0x8 logical shards); then the GPU suites of the paths touched
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05f; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["config"].get("rows"), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("oracle_check", {}).get("ok"), d.get("phases_ms"))'
timeout -k 10 300 python -u bench.py > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
python3 -c "$S" < $O/bench_cfg3.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
python3 -c "$S" < $O/bench_shard_fc.log
timeout -k 10 300 python -u bench.py --rows 100000 --dtype f32 --nq 1 --steps 2000 --warmup 200 --event-stride 16 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { tail -30 $O/bench_cfg2.log; exit 1; }
python3 -c "$S" < $O/bench_cfg2.log
timeout -k 10 300 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --no-cpu-baseline --steps 20 --warmup 3 --oracle-stride 4 > $O/bench_cfg4.log 2>&1 || { tail -20 $O/bench_cfg4.log; exit 1; }
python3 -c "$S" < $O/bench_cfg4.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg3_b.log 2>&1 || { tail -30 $O/bench_cfg3_b.log; exit 1; }
python3 -c "$S" < $O/bench_cfg3_b.log
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc_b.log 2>&1 || { tail -30 $O/bench_shard_fc_b.log; exit 1; }
python3 -c "$S" < $O/bench_shard_fc_b.log
timeout -k 10 400 python -u tools/sharded_host_issue.py --rows 10000000 --devices 0x8 > $O/sharded_host_issue.json 2>&1 || { tail -30 $O/sharded_host_issue.json; exit 1; }
grep -v amdgpu $O/sharded_host_issue.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kts -o kts -- python $R/bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_kts.log 2>&1 || { tail -20 $O/bench_kts.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt2 -- python $R/bench.py --rows 100000 --dtype f32 --nq 1 --steps 300 --warmup 20 --event-stride 16 --no-cpu-baseline > $O/bench_kt2.log 2>&1 || { tail -20 $O/bench_kt2.log; exit 1; }
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_screen_valu.py tests/test_gpu_fused.py tests/test_gpu_screen.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_screen_capacity.py tests/test_gpu_union.py tests/test_gpu_filters.py tests/test_gpu_merge.py tests/test_gpu_bench_rehearsal.py > $O/pytest_paths.log 2>&1 || { tail -40 $O/pytest_paths.log; exit 1; }
tail -3 $O/pytest_paths.log
