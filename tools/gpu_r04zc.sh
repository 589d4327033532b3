#!/bin/bash
# round 4: box-to-box check of the final build: the default bench twice and kernel 10 balanced vs static
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04zc; mkdir -p $O
for i in 1 2; do
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $O/bench_default_$i.log 2>&1 || { tail -30 $O/bench_default_$i.log; exit 1; }
tail -1 $O/bench_default_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['oracle_check']['ok'])"
done
timeout -k 10 300 python -u tools/k10_variants.py --rows 10000000 --variants 800000,804096 --rounds 6 --burst 30 > $O/k10_10m_ab.txt 2>&1 || { tail -20 $O/k10_10m_ab.txt; exit 1; }
grep -v amdgpu $O/k10_10m_ab.txt | tr -d ' \n'; echo
