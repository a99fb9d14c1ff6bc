#!/usr/bin/env python3
"""Per-queue busy time and the dispatch timeline of the last full training step in a rocprofv3
kernel trace (the step = dispatches after the second-to-last adam_kernel / adam_t_kernel up to the last).

  python scripts/step_timeline.py <k_kernel_trace.csv> [first last]   # print dispatches first..last
"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = re.sub(r"^void ", "", r["Kernel_Name"]).replace("pvr::(anonymous namespace)::", "")
        r["n"] = n.split("(")[0][:48]
    rows.sort(key=lambda r: r["s"])
    ad = [i for i, r in enumerate(rows) if "adam_kernel" in r["n"] or "adam_t_kernel" in r["n"]]
    step = rows[ad[-2] + 1: ad[-1] + 1]
    t0, t1 = step[0]["s"], step[-1]["e"]
    print(f"step {(t1 - t0) / 1e6:.3f} ms, {len(step)} dispatches")
    for q in sorted({r["Queue_Id"] for r in step}):
        rs = [r for r in step if r["Queue_Id"] == q]
        print(f"queue {q}: {len(rs)} dispatches, busy {sum(r['e'] - r['s'] for r in rs) / 1e6:.3f} ms")
    lo, hi = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (0, len(step))
    print("queue | kernel | start us | dur us | grid")
    for r in step[lo:hi]:
        grid = r.get("Grid_Size_X", r.get("Grid_Size", ""))
        print(f"{r['Queue_Id']} | {r['n']} | {(r['s'] - t0) / 1e3:.1f} | {(r['e'] - r['s']) / 1e3:.1f} | {grid}")


if __name__ == "__main__":
    main()
