#!/bin/bash
# round 3: kernel-10 ablations and ring depths (debug library), config 3 shape
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u tools/k10_variants.py > gpurun_out/r03c_k10_variants.json 2> gpurun_out/r03c_k10_variants.err
rc=$?
cat gpurun_out/r03c_k10_variants.json; tail -5 gpurun_out/r03c_k10_variants.err
exit $rc
