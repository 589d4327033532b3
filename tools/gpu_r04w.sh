#!/bin/bash
# round 4: kernel 10 with the XCD-balanced tile split: correctness (two-pass tests incl. the full-size
# 10M oracle check), block tails balanced vs static, interleaved timing A/B, the shard step and config 3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"], d.get("oracle_check",{}).get("ok"))'
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_screen.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py tests/test_gpu_screen_capacity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 865536 869632; do
timeout -k 10 300 python -u tools/k10_block_times.py --rows 10000000 --reps 12 --variant $v > $O/k10_block_times_10m_$v.json 2>&1 || { tail -20 $O/k10_block_times_10m_$v.json; exit 1; }
grep -v amdgpu $O/k10_block_times_10m_$v.json | tr -d ' \n'; echo
done
timeout -k 10 300 python -u tools/k10_variants.py --rows 10000000 --variants 800000,804096 --rounds 6 --burst 30 > $O/k10_10m_ab.txt 2>&1 || { tail -20 $O/k10_10m_ab.txt; exit 1; }
grep -v amdgpu $O/k10_10m_ab.txt | tr -d ' \n'; echo
timeout -k 10 240 python -u tools/k10_variants.py --rows 1250000 --variants 800000,804096 --rounds 8 --burst 100 > $O/k10_shard_ab.txt 2>&1 || { tail -20 $O/k10_shard_ab.txt; exit 1; }
grep -v amdgpu $O/k10_shard_ab.txt | tr -d ' \n'; echo
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_shard_fc.log 2>&1 || { tail -30 $O/bench_shard_fc.log; exit 1; }
tail -1 $O/bench_shard_fc.log | python3 -c "$S"
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
