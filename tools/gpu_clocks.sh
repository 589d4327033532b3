#!/bin/bash
# Steady state under the power cap: each variant runs back to back for ~8 s while rocm-smi samples
# package power and sclk mid-run; the variant's per-launch time is the burst average.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/clocks"
rm -rf "$O"; mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
for m in ${CMODES:-20000000 20000016 20000032 20000048 132072 20000009 20000041 1003}; do
  timeout -k 10 200 python -u tools/k5_variants.py --modes $m --rounds 1 --burst 2000 --warm-seconds 1 --no-stream-ref > "$O/run_$m.json" 2> "$O/run_$m.err" &
  pid=$!
  sleep 9
  for i in 1 2 3; do timeout -k 5 20 rocm-smi --showclocks --showpower >> "$O/smi_$m.txt" 2>&1; sleep 0.5; done
  wait $pid || { echo "run $m failed"; tail -5 "$O/run_$m.err"; exit 1; }
  echo "$m $(tail -1 $O/run_$m.json | cut -c1-90) | $(grep -oE 'sclk clock level: [0-9]: \([0-9]+Mhz\)|Power \(W\): [0-9.]+' $O/smi_$m.txt | tr '\n' ' ')"
done
