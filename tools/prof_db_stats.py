"""Dev tool: write the per-kernel summary (name, calls, total ns, average ns, percent) of a
rocprofv3 SQLite database (run_results.db, the tool's default output format) as CSV — the same
columns as rocprofv3 --stats --output-format csv's kernel_stats.csv.
Usage: python tools/prof_db_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, total, avg, pct in c.execute("select name, total_calls, total_duration, average, percentage "
                                                  "from top_kernels order by total_duration desc"):
        w.writerow([name, calls, round(total, 3), round(avg, 3), round(pct, 4)])
