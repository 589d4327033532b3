#!/bin/bash
# Round 6: the -m gpu suite without the full-size files, then the benches this round's changes touch
# (padded 2-wave batches, config 3 with virtual-memory rows, kernel 10 with 64 queries per wave, the sharded
# issue pool).
set -o pipefail
O=${1:-gpurun_out/r06b}
mkdir -p "$O"
export TMPDIR=/tmp
tools/r06/gpu_tests.sh "$O" tests --ignore tests/test_gpu_fullsize.py \
  --ignore tests/test_gpu_ivf_cfg5.py --ignore tests/test_gpu_ivf_4m.py || exit 1
for nq in 16 32; do
  timeout -k 10 300 python -u bench.py --nq $nq --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_10m_nq${nq}_auto.log" 2>&1 || { echo "bench nq=$nq rc=$?"; exit 1; }
  tail -1 "$O/bench_10m_nq${nq}_auto.log" | cut -c1-200
done
timeout -k 10 400 python -u bench.py > "$O/bench_default.log" 2>&1 || { echo "bench default rc=$?"; exit 1; }
tail -1 "$O/bench_default.log" | cut -c1-300
RFX_K10_Q64=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench_default_q64.log" 2>&1 || { echo "bench q64 rc=$?"; tail -5 "$O/bench_default_q64.log"; exit 1; }
tail -1 "$O/bench_default_q64.log" | cut -c1-300
for v in 0 1; do
  RFX_K10_Q64=$v timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --no-cpu-baseline --steps 50 > "$O/bench_shard_q64_$v.log" 2>&1 || { echo "bench shard q64=$v rc=$?"; tail -5 "$O/bench_shard_q64_$v.log"; exit 1; }
  tail -1 "$O/bench_shard_q64_$v.log" | cut -c1-200
done
RFX_ISSUE_THREADS=0 timeout -k 10 300 python -u tools/sharded_host_issue.py > "$O/sharded_host_issue_serial.json" 2> "$O/sharded_host_issue.err" || { echo "host issue rc=$?"; tail -5 "$O/sharded_host_issue.err"; exit 1; }
timeout -k 10 300 python -u tools/sharded_host_issue.py > "$O/sharded_host_issue.json" 2>> "$O/sharded_host_issue.err" || { echo "host issue rc=$?"; tail -5 "$O/sharded_host_issue.err"; exit 1; }
cat "$O/sharded_host_issue_serial.json" "$O/sharded_host_issue.json"
