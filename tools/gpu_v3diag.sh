#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for nq in 128 256; do
  timeout -k 10 200 python tools/scan_variants.py --nq $nq --modes 3 > gpurun_out/v3_nq$nq.json 2> gpurun_out/v3.err || { echo "variants rc=$?"; tail -5 gpurun_out/v3.err; exit 1; }
  echo "nq=$nq $(cat gpurun_out/v3_nq$nq.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc3 -o pmc -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc3.log 2>&1 || { echo "pmc rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc3.log; exit 1; }
grep -h scan_mfma3 $GRAFT_REPO_ROOT/gpurun_out/pmc3/pmc_counter_collection.csv | awk -F, '{print $(NF-2), $(NF-3)}' | head -4
