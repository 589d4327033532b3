#!/bin/bash
# round 3: kernel 11 phase ablations at config 2 (RFX_K11_ABLATE bits: 2 no row stream, 4 no query
# quantiser, 8 no last-block select; timing only), then parity tests and the checked bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03q; mkdir -p $O
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 2000 --warmup 50 --event-stride 16 --no-cpu-baseline"
for m in 0 8 16; do
  RFX_K11_ABLATE=$m timeout -k 10 200 python -u bench.py $C2 --oracle-stride 0 > $O/bench_ab$m.log 2>&1 || { tail -20 $O/bench_ab$m.log; exit 1; }
  echo "ablate $m: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_ab$m.log) $(grep -o '"kernel_ms": [0-9.]*' $O/bench_ab$m.log)"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen_valu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u bench.py $C2 > $O/bench_cfg2.log 2>&1 || { tail -20 $O/bench_cfg2.log; exit 1; }
tail -c 1500 $O/bench_cfg2.log
