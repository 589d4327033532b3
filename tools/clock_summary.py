"""Summarise a rocprofv3 --pmc GRBM_GUI_ACTIVE pass: effective clock per kernel dispatch
(GRBM_GUI_ACTIVE / 8 XCDs / wall), grouped by kernel name.  Dev tool, not product."""
import collections
import csv
import glob
import os
import sys

rows = collections.defaultdict(dict)
for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (r["Dispatch_Id"], r["Kernel_Name"])
            rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[key]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
agg = collections.defaultdict(list)
for (did, name), d in sorted(rows.items(), key=lambda kv: int(kv[0][0])):
    if "GRBM_GUI_ACTIVE" in d and d["ns"] > 3e5:
        short = name.split("(")[0][-60:]
        agg[short].append((int(did), d["ns"] / 1e6, d["GRBM_GUI_ACTIVE"] / 8 / d["ns"], d.get("SQ_BUSY_CYCLES", 0),
                           d.get("SQ_WAVE_CYCLES", 0)))
for k, v in agg.items():
    for did, ms, ghz, busy, wc in v[-12:]:
        print(f"{did:5d} {k:60s} {ms:8.3f} ms  {ghz:5.2f} GHz  wave_cyc {wc:.3e}")
