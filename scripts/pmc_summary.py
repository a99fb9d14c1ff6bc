#!/usr/bin/env python3
"""Per-kernel mean of every rocprofv3 --pmc counter found under a directory (counter_collection CSVs
of scripts/pmc_attn.sh passes), plus the mean kernel duration from the kernel traces; markdown."""
from __future__ import annotations

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("pvr::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)[:70]


def grid_tag(r) -> str:
    """' [grid N]' when the CSV row carries a grid size (tells shapes of one kernel variant apart)"""
    for col in ("Grid_Size", "Grid_Size_X"):
        if r.get(col):
            return f" [grid {r[col]}]"
    return ""


def main():
    root = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"]) + grid_tag(r)
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"]) + grid_tag(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "attn")
    for k in sorted(vals):
        if not pat.search(k):
            continue
        d = dur.get(k, [])
        print(f"## {k}\n\nmean duration {sum(d) / max(len(d), 1):.1f} us over {len(d)} dispatches\n")
        print("| counter | mean per dispatch |\n|---|---:|")
        for c in sorted(vals[k]):
            v = vals[k][c]
            print(f"| {c} | {sum(v) / len(v):,.0f} |")
        print()


if __name__ == "__main__":
    main()
