#!/bin/bash
# round 3: kernel 11 with the 16-slot bound: parity tests, config-2 benches (two-pass / exact), rocprof
# kernel stats of the two-pass config-2 run; the 2-rank gloo rehearsal with --check
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen_valu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 2000 --warmup 50 --event-stride 16 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2.log 2>&1 || { tail -20 $O/bench_cfg2.log; exit 1; }
tail -c 1800 $O/bench_cfg2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python -u bench.py $C2 --oracle-stride 0 > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
find $O/prof2 -name "*kernel_stats.csv" -exec head -6 {} \; | cut -c1-150
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --one-device --check > $O/rehearsal2.log 2>&1 || { tail -20 $O/rehearsal2.log; exit 1; }
grep -E "check ok|\"metric\"" $O/rehearsal2.log | cut -c1-2500
