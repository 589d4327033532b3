#!/bin/bash
# round 3: after the launder fix — kernel-10 variants, then cfg3 bench two-pass and exact
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u tools/k10_variants.py > gpurun_out/r03d_k10_variants.json 2> gpurun_out/r03d_k10_variants.err || { tail -5 gpurun_out/r03d_k10_variants.err; exit 1; }
cat gpurun_out/r03d_k10_variants.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03d_bench_screen.log 2>&1 || { tail -20 gpurun_out/r03d_bench_screen.log; exit 1; }
tail -c 2500 gpurun_out/r03d_bench_screen.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --scan exact --no-cpu-baseline > gpurun_out/r03d_bench_exact.log 2>&1 || { tail -20 gpurun_out/r03d_bench_exact.log; exit 1; }
tail -c 1800 gpurun_out/r03d_bench_exact.log
