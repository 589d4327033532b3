#!/bin/bash
# round 3: kernel 10's slow path with a chain-free list insert (independent compares) and the pass
# mask's live bits applied once — variants at config 3 (10M) and at the 8-GPU shard (1.25M), the
# two-pass tests, config-3 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 300 python -u tools/k10_variants.py --variants 8000,9024,8512 --rounds 4 > $O/k10_10m.txt 2>&1 || { tail -20 $O/k10_10m.txt; exit 1; }
timeout -k 10 300 python -u tools/k10_variants.py --rows 1250000 --variants 8000,9024,8512 --rounds 6 --burst 100 > $O/k10_shard.txt 2>&1 || { tail -20 $O/k10_shard.txt; exit 1; }
grep -A3 '"8000"\|"9024"\|"8512"' $O/k10_10m.txt $O/k10_shard.txt | grep min
timeout -k 10 600 python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -c 1500 $O/bench.log
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt3 -o kt -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --oracle-stride 0 > $R/$O/bench_prof3.log 2>&1 || { tail -20 $R/$O/bench_prof3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kts -o kt -- python $R/bench.py --rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --oracle-stride 0 --force-comm > $R/$O/bench_shard_fc.log 2>&1 || { tail -20 $R/$O/bench_shard_fc.log; exit 1; }
tail -c 700 $R/$O/bench_shard_fc.log
