#!/bin/bash
# Effective clock per scan variant: rocprofv3 PMC GRBM_GUI_ACTIVE (summed over 8 XCDs) / 8 / dispatch
# wall time (MI355X_MICROARCH.md 'DVFS give-back').  One PMC pass; no tracing domains.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
rm -rf "$O/prof_clk"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$O/prof_clk" -o clk -- python "$R/tools/scan_variants.py" --rounds 3 --warm-seconds 1 --modes ${MODES:-3,21,23,29} > "$O/clk.log" 2>&1 || { echo "clk rc=$?"; tail -20 "$O/clk.log"; exit 1; }
tail -1 "$O/clk.log"
python "$R/tools/clock_summary.py" "$O/prof_clk"
