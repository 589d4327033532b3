#!/bin/bash
# round 3: kernel-10 variants in 8-s steady bursts with rocm-smi power / sclk samples
# (800 production, 928 epilogue in place, 801 no fold, 809 no fold + no stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03n; mkdir -p $O
for v in 800 928 801 809; do
  timeout -k 10 120 python -u tools/k10_variants.py --variants $v --seconds 16 > $O/run_$v.json 2> $O/run_$v.err &
  pid=$!
  sleep 12
  for i in 1 2 3; do timeout -k 5 20 rocm-smi --showclocks --showpower >> $O/smi_$v.txt 2>&1; sleep 0.5; done
  wait $pid || { echo "run $v failed"; tail -5 $O/run_$v.err; exit 1; }
  echo "$v $(cat $O/run_$v.json) | $(grep -oE 'sclk clock level: [0-9]+: \([0-9]+Mhz\)|Power \(W\): [0-9.]+' $O/smi_$v.txt | tr '\n' ' ')"
done
