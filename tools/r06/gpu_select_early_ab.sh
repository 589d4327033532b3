#!/bin/bash
# Round 6: the select with every kept candidate's row loaded before a_k (k_select.h early path) against
# the previous build (librfx_base.so): the two-pass GPU tests, then the 8-GPU shard step and config 3
# interleaved, then rocprof kernel traces of the shard step for both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06sel}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_screen_w2.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_screen_capacity.py > $O/pytest_sel.log 2>&1 || { tail -40 $O/pytest_sel.log; exit 1; }
tail -1 $O/pytest_sel.log
for v in new base; do
  L=librfx_dbg.so; [ $v = base ] && L=librfx_dbg_base.so
  RFX_LIB=$R/rag-foundation_amd/rfx/$L RFX_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u tools/select_phases.py --rows 1250000 > $O/phases_shard_$v.json 2> $O/phases_shard_$v.err || { tail -20 $O/phases_shard_$v.err; exit 1; }
  echo "phases shard $v: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['median_rep']; print(d['span_ns'], d['block_ns_med'], d['block_ns_max'], d['phase_ns_med'], d['phase_ns_max'])" $O/phases_shard_$v.json)"
done
for v in new base; do
  if [ $v = base ]; then export RFX_LIB=$R/rag-foundation_amd/rfx/librfx_base.so RFX_ALLOW_STALE_LIB=1; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o kt_$v -- python $R/bench.py --rows 1250000 --force-comm --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_kt_$v.log 2>&1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3_$v -o kt3_$v -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_kt3_$v.log 2>&1 || { tail -20 $O/bench_kt_$v.log; exit 1; }
  cp $(ls $O/kt_$v/*kernel_stats.csv) $O/kt_${v}_kernel_stats.csv && cp $(ls $O/kt3_$v/*kernel_stats.csv) $O/kt3_${v}_kernel_stats.csv
  python3 -c "import csv,sys; [print('$v', f, r[0][:50], r[1], r[3]) for f in sys.argv[1:] for r in csv.reader(open(f)) if 'select' in r[0] or 'scan_screen' in r[0]]" $O/kt_${v}_kernel_stats.csv $O/kt3_${v}_kernel_stats.csv
done
