#!/bin/bash
# Profiling session: scan ablations, rocprofv3 kernel stats of the bench, then a separate PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python tools/scan_variants.py > gpurun_out/variants.json 2> gpurun_out/variants.err || { echo "variants rc=$?"; tail -20 gpurun_out/variants.err; exit 1; }
cat gpurun_out/variants.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_kt -o kt -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_kt.log 2>&1 || { echo "kt rc=$?"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bench_kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_pmc -o pmc -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bench_pmc.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_kt $GRAFT_REPO_ROOT/gpurun_out/prof_pmc -type f | head -20
