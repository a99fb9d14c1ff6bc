#!/usr/bin/env python3
"""Kernel time of ONE steady-state training step from a rocprofv3 kernel trace (the kernels between
the last two Adam launches), grouped by kernel: markdown table.

  python scripts/steady_step.py gpurun_out/final1/h14_prof/step_kernel_trace.csv "ViT-H/14 fp8 b256"
"""
import collections
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].replace("pvr::(anonymous namespace)::", "") for r in rows]
    idx = [i for i, n in enumerate(names) if "adam" in n]
    a, b = idx[-2], idx[-1]
    cnt, tot = collections.Counter(), collections.Counter()
    for j in range(a + 1, b + 1):
        k = names[j].split("(")[0].replace("void ", "")[:70]
        cnt[k] += 1
        tot[k] += (int(rows[j]["End_Timestamp"]) - int(rows[j]["Start_Timestamp"])) / 1e6
    s = sum(tot.values())
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e6
    print(f"# {title}: one steady-state step (serial weight gradients)\n")
    print(f"Kernel time {s:.2f} ms, wall {wall:.2f} ms, {sum(cnt.values())} launches.\n")
    print("| kernel | launches | ms | % |\n|---|---:|---:|---:|")
    for k, v in tot.most_common():
        print(f"| `{k}` | {cnt[k]} | {v:.3f} | {100 * v / s:.1f} |")


if __name__ == "__main__":
    main()
