#!/bin/bash
# round 3: kernel 10's list in registers for the whole scan (no LDS list in production), select's
# survivor-row array — variants at config 3 (10M) and the 8-GPU shard (1.25M), smoke, the full -m gpu
# suite, config-3 bench, rocprof stats (config 3, shard through the 1-rank RCCL step)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --variants 8000,9024,8512 --rounds 4 > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 8000,9024,8512 --rounds 6 --burst 100 > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -A3 '"8000"\|"9024"\|"8512"' $O/k10_10m.txt $O/k10_shard.txt | grep min
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt3 -o kt -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --oracle-stride 0 > $R/$O/bench_prof3.log 2>&1 || { tail -20 $R/$O/bench_prof3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kts -o kt -- python $R/bench.py --rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0 --force-comm > $R/$O/bench_shard_fc.log 2>&1 || { tail -20 $R/$O/bench_shard_fc.log; exit 1; }
echo done
