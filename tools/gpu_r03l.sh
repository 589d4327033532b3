#!/bin/bash
# round 3: per-tile-scale fast path in kernel 10 (A/B against the store-wide bound), sharded IVF +
# device-to-device re-split tests, config-3 and config-4-shard benches (two-pass and exact)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_screen.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/k10_variants.py --variants 832,896,800,864,801 --rounds 4 > $O/variants.json 2> $O/variants.err || { tail -5 $O/variants.err; exit 1; }
cat $O/variants.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -c 2500 $O/bench_cfg3.log
timeout -k 10 300 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg4.log 2>&1 || { tail -20 $O/bench_cfg4.log; exit 1; }
tail -c 2500 $O/bench_cfg4.log
timeout -k 10 300 python -u bench.py --rows 12500000 --dim 1024 --dtype f16 --steps 20 --warmup 3 --scan exact --no-cpu-baseline --oracle-stride 0 > $O/bench_cfg4_exact.log 2>&1 || { tail -20 $O/bench_cfg4_exact.log; exit 1; }
tail -c 1500 $O/bench_cfg4_exact.log
