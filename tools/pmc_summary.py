"""Dev tool: per-kernel averages of rocprofv3 --pmc counter CSVs (one or more passes).

usage: python tools/pmc_summary.py <counter_collection.csv> [...] [--kernel SUBSTR] [--json OUT]
Prints, per kernel name (template arguments kept, so MODE variants separate), the mean of every counter
over its dispatches, and the derived ratios used in DESIGN §4.10 (SQ_* cycle counters are per-XCD sums
of quad-cycles: only their ratios are compared)."""
import argparse
import collections
import csv
import json


def load(paths, substr):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                if substr and substr not in row["Kernel_Name"]:
                    continue
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} | {"_dispatches": max(len(v) for v in d.values())}
            for k, d in acc.items()}


def derived(c):
    out = {}
    g = c.get
    if g("SQ_WAVE_CYCLES"):
        w = g("SQ_WAVE_CYCLES")
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
            if g(n) is not None:
                out[n + "/WAVE_CYCLES"] = round(g(n) / w, 4)
    if g("SQ_BUSY_CYCLES") and g("SQ_VALU_MFMA_BUSY_CYCLES"):
        out["MFMA_BUSY/BUSY_CYCLES"] = round(g("SQ_VALU_MFMA_BUSY_CYCLES") / g("SQ_BUSY_CYCLES"), 4)
    if g("SQ_INSTS_MFMA"):
        m = g("SQ_INSTS_MFMA")
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"):
            if g(n) is not None:
                out[n + "/MFMA"] = round(g(n) / m, 4)
    if g("SQ_LDS_IDX_ACTIVE") and g("SQ_LDS_BANK_CONFLICT") is not None:
        out["LDS_BANK_CONFLICT/LDS_IDX_ACTIVE"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--json")
    a = ap.parse_args()
    res = load(a.csv, a.kernel)
    out = {k: {"counters": v, "derived": derived(v)} for k, v in res.items()}
    for k, v in out.items():
        print(k[:110])
        for c, x in sorted(v["counters"].items()):
            print(f"  {c:32s} {x:.6g}")
        for c, x in v["derived"].items():
            print(f"  {c:40s} {x}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
