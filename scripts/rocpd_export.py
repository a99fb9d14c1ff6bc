#!/usr/bin/env python3
"""Export a rocprofv3 SQLite (rocpd) database to the CSV layouts the other profile tools read.

usage: rocpd_export.py <results.db> <out_prefix>
  writes <out_prefix>_kernel_trace.csv (Kernel_Name, Start_Timestamp, End_Timestamp, Stream_Id)
     and <out_prefix>_kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage)
"""
import csv
import sqlite3
import sys


def main():
    db, prefix = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    with open(prefix + "_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"])
        w.writerows(rows)
    agg = {}
    for name, s, e, _ in rows:
        n, t = agg.get(name, (0, 0))
        agg[name] = (n + 1, t + (e - s))
    total = sum(t for _, t in agg.values()) or 1
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, n, t, t / n, 100.0 * t / total])
    print(f"{len(rows)} dispatches, {len(agg)} kernels -> {prefix}_kernel_{{trace,stats}}.csv")


if __name__ == "__main__":
    main()
