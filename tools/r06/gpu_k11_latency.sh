#!/bin/bash
# Round 6: kernel 11's per-search latency alone, beside a stream of kernel-10 batches, and with two
# kernel-11 streams at once (ordered by librfx, then unordered) — tools/k11_latency.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/r06lat}; mkdir -p $O
timeout -k 10 300 python -u tools/k11_latency.py > $O/k11_latency_ordered.json 2> $O/k11_latency_ordered.err || { tail -20 $O/k11_latency_ordered.err; exit 1; }
cat $O/k11_latency_ordered.json
RFX_K11_UNORDERED=1 timeout -k 10 300 python -u tools/k11_latency.py > $O/k11_latency_unordered.json 2> $O/k11_latency_unordered.err || { tail -20 $O/k11_latency_unordered.err; exit 1; }
cat $O/k11_latency_unordered.json
