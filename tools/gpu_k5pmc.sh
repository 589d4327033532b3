#!/bin/bash
# PMC passes over the headline kernel and its no-stream / no-MFMA ablations (debug library).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/k5pmc"
mkdir -p "$O"
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+|GRBM_[A-Z_]+|TCP_[A-Z0-9_]+|TA_[A-Z0-9_]+" "$O/counters.txt" | sort -u > "$O/counter_names.txt"
MODES="--modes ${PMODES:-132072,20000000,20000009,1009,1003} --rounds 1 --burst 3 --warm-seconds 1"
i=0
run() {
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $1 --output-format csv -d "$O/p$i" -o p$i -- python "$R/tools/k5_variants.py" $MODES > "$O/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -5 "$O/p$i.log"; return 1; }
}
run "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" && \
run "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" && \
run "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
python - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        kn = r["Kernel_Name"]
        if "scan_mfma5" not in kn and "scan_mfma6" not in kn:
            continue
        mode = ("k5:" if "scan_mfma5" in kn else "k6:") + kn.split("_kernel<")[1].split(">")[0].split(",")[-1].strip()
        agg[mode][r["Counter_Name"]].append(float(r["Counter_Value"]))
for m, d in agg.items():
    print(m, {k: round(sum(v) / len(v) / 1e6, 3) for k, v in sorted(d.items())})
PY
