#!/bin/bash
# round 4 (r04k): event overhead of the N > 1 step (events every step vs once), host issue time, kernel 11
# phases at config 2, the config-3 default step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
S='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["config"]["workload"][:30], d["ms_per_step"], d.get("host_issue_ms_per_step"), d["phases_ms"], d["roofline"]["kernel_ms"])'
for es in 1 1000; do
timeout -k 10 300 python -u bench.py --rows 1250000 --force-comm --steps 400 --warmup 20 --no-cpu-baseline --event-stride $es > $O/bench_shard_es$es.log 2>&1 || { tail -30 $O/bench_shard_es$es.log; exit 1; }
tail -1 $O/bench_shard_es$es.log | python3 -c "$S"
done
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 400 --warmup 20 --no-cpu-baseline --event-stride 1000 > $O/bench_shard_nocomm.log 2>&1 || { tail -30 $O/bench_shard_nocomm.log; exit 1; }
tail -1 $O/bench_shard_nocomm.log | python3 -c "$S"
timeout -k 10 300 python -u tools/k11_phases.py > $O/k11_phases.json 2>&1 || { tail -20 $O/k11_phases.json; exit 1; }
cat $O/k11_phases.json | tr -d ' \n'; echo
timeout -k 10 420 python -u bench.py > $O/bench_cfg3.log 2>&1 || { tail -30 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | python3 -c "$S"
