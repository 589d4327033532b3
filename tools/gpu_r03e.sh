#!/bin/bash
# round 3: kernel 6 with / without the launder of its resident fragments, same box, interleaved bursts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u tools/k5_variants.py --modes 20000000,20001024 --no-stream-ref --rounds 6 > gpurun_out/r03e_k6_launder.json 2> gpurun_out/r03e_k6_launder.err || { tail -5 gpurun_out/r03e_k6_launder.err; exit 1; }
tail -40 gpurun_out/r03e_k6_launder.json
