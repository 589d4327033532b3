"""Turn rocprofv3 PMC / kernel-trace CSVs of a bench run into profiles/ summaries.

FETCH_SIZE (KB) on gfx950 counts 64 B per TCC_EA0_RDREQ while a wide coalesced stream issues
128-B requests, i.e. it reads half the bytes (MI355X_MICROARCH.md §HBM): hbm read bytes =
2 × FETCH_SIZE × 1024.  WRITE_SIZE reads exactly for 16-B streaming stores.  The per-launch
traffic of the scan kernel is the average over its dispatches.

usage: python tools/collect_pmc.py <fetch_csv> [<write_csv>] --key WORKLOAD --kernel SUBSTR
       [--stats KT_STATS_CSV] --out profiles/pmc_traffic.json
"""
import argparse
import csv
import json
import os


def per_kernel(path, counter, substr):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and substr in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv", nargs="?")
    ap.add_argument("--key", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_csv, "FETCH_SIZE", a.kernel)
    if not fetch:
        raise SystemExit(f"no FETCH_SIZE rows for kernel matching {a.kernel!r}")
    read_b = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    write_b = None
    if a.write_csv:
        w = per_kernel(a.write_csv, "WRITE_SIZE", a.kernel)
        write_b = 1024.0 * sum(w) / len(w) if w else None
    entry = {"kernel_match": a.kernel, "dispatches": len(fetch),
             "fetch_size_kb_avg": sum(fetch) / len(fetch),
             "hbm_read_bytes_per_launch": read_b,
             "hbm_write_bytes_per_launch": write_b,
             "hbm_bytes_per_launch": read_b + (write_b or 0.0),
             "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 counts 64 B per 128-B request)"}
    if a.stats:
        with open(a.stats) as f:
            for row in csv.DictReader(f):
                if a.kernel in row["Name"]:
                    entry["kernel_avg_ns"] = float(row["AverageNs"])
                    entry["kernel_calls"] = int(row["Calls"])
    d = {}
    if os.path.exists(a.out):
        d = json.load(open(a.out))
    d[a.key] = entry
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps({a.key: entry}))


if __name__ == "__main__":
    main()
