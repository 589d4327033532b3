#!/bin/bash
# round 3: kernel 10 with the KL-th-largest-of-16 slot bound vs the min-of-KL bound; gather exchange;
# full GPU test files touched this round; bench cfg3 (+ 1-rank RCCL step, gloo rehearsal)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_screen_valu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/k10_variants.py --variants 8032,8288,8000,8256,8512,8001 --rounds 4 > $O/variants.json 2> $O/variants.err || { tail -5 $O/variants.err; exit 1; }
cat $O/variants.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -c 2500 $O/bench_cfg3.log
C2="--rows 100000 --dim 768 --dtype f32 --nq 1 --k 10 --steps 2000 --warmup 50 --event-stride 16 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C2 > $O/bench_cfg2.log 2>&1 || { tail -20 $O/bench_cfg2.log; exit 1; }
tail -c 1800 $O/bench_cfg2.log
timeout -k 10 300 python -u bench.py $C2 --scan exact --oracle-stride 0 > $O/bench_cfg2_exact.log 2>&1 || { tail -20 $O/bench_cfg2_exact.log; exit 1; }
tail -c 1200 $O/bench_cfg2_exact.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-comm --oracle-stride 16 > $O/bench_cfg3_comm1.log 2>&1 || { tail -20 $O/bench_cfg3_comm1.log; exit 1; }
tail -c 1500 $O/bench_cfg3_comm1.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --one-device --check > $O/rehearsal2.log 2>&1 || { tail -20 $O/rehearsal2.log; exit 1; }
grep -E "check ok|\"metric\"" $O/rehearsal2.log | cut -c1-2500
