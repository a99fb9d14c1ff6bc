#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV into a markdown table (per-step ms per kernel).

usage: summarize_prof.py <kernel_stats.csv> <steps_profiled> [title]
"""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"pvr::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(pvr::GemmParams\)", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    name = name.replace("void ", "")
    return name[:110]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    title = sys.argv[3] if len(sys.argv) > 3 else path
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Total GPU kernel time over the profiled run: {total / 1e6:.1f} ms "
          f"({steps} profiled steps incl. warmup -> {total / 1e6 / steps:.2f} ms/step upper bound)\n")
    print("| kernel | calls | total ms | ms/step | % | avg us |")
    print("|---|---:|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {t / 1e6:.2f} | {t / 1e6 / steps:.3f} | "
              f"{100 * t / total:.1f} | {float(r['AverageNs']) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
