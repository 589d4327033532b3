#!/bin/bash
# Sample the SMU's clocks and power (rocm-smi) while the headline kernel runs back to back, and
# while the stream-only / MFMA-only ablations run: is the memory side throttled under MFMA load?
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/clocks"
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 5 20 rocm-smi --showclocks --showpower > "$O/idle.txt" 2>&1
for m in 20000000 1003 20000009; do
  timeout -k 10 200 python -u tools/k5_variants.py --modes $m --rounds 1 --burst 3000 --warm-seconds 1 > "$O/run_$m.json" 2> "$O/run_$m.err" &
  pid=$!
  sleep 12
  for i in 1 2 3; do timeout -k 5 20 rocm-smi --showclocks --showpower >> "$O/smi_$m.txt" 2>&1; sleep 1; done
  wait $pid || { echo "run $m failed"; tail -5 "$O/run_$m.err"; exit 1; }
  tail -1 "$O/run_$m.json"
done
grep -hE "fclk|mclk|sclk|socclk|Power" "$O"/smi_*.txt | head -60
