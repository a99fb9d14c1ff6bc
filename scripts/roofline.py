#!/usr/bin/env python3
"""Per-kernel roofline table of one training step from scripts/gpu_roofline.sh output.

Inputs (all with the weight-gradient side stream off, so dispatches are serial and in a fixed order):
  trace/k_kernel_trace.csv         kernel times (no counters: undisturbed durations)
  pmc1 FETCH_SIZE, pmc2 WRITE_SIZE, pmc3 SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE
The last complete step of each run (dispatches after the second-to-last adam_kernel up to the last)
is aligned position by position (kernel names must match).

Derived per dispatch:
  FLOP      = SQ_VALU_MFMA_BUSY_CYCLES * 1024 (bf16 MFMA: 16x16x32 = 16 cycles, 32x32x16 = 32 cycles,
              i.e. 1024 FLOP per busy cycle on a SIMD)
  MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
  HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB; gfx950 FETCH_SIZE counts half of a wide coalesced
              stream's bytes, MI355X_MICROARCH.md) -> an upper estimate of read bytes
Roofline bound = max(FLOP / 2.5 PF, bytes / 8 TB/s); "% of bound" = bound / measured time.
Usage: python scripts/roofline.py gpurun_out/roof > profiles/.../roofline.md
"""
from __future__ import annotations

import collections
import csv
import os
import re
import sys

PEAK_FLOPS = 2.5e15
PEAK_BW = 8.0e12


def short(n: str) -> str:
    n = re.sub(r"^void ", "", n).replace("pvr::(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def last_step(rows):
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    return rows[ad[-2] + 1: ad[-1] + 1]


def load_trace(path):
    return last_step(list(csv.DictReader(open(path))))


def load_pmc(path):
    by = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = by.setdefault(r["Dispatch_Id"], dict(r, counters={}))
        d["counters"][r["Counter_Name"]] = float(r["Counter_Value"])
    return last_step(list(by.values()))


def main():
    root = sys.argv[1]
    tr = load_trace(os.path.join(root, "trace", "k_kernel_trace.csv"))
    p1 = load_pmc(os.path.join(root, "pmc1", "p_counter_collection.csv"))
    p2 = load_pmc(os.path.join(root, "pmc2", "p_counter_collection.csv"))
    p3 = load_pmc(os.path.join(root, "pmc3", "p_counter_collection.csv"))
    n = min(len(tr), len(p1), len(p2), len(p3))
    groups = collections.OrderedDict()
    step_us = 0.0
    for i in range(n):
        t, a, b, c = tr[i], p1[i], p2[i], p3[i]
        names = {short(x["Kernel_Name"]) for x in (t, a, b, c)}
        if len(names) != 1:
            raise SystemExit(f"dispatch {i}: sequences differ: {names}")
        dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3  # us
        step_us += dur
        busy = c["counters"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gui = c["counters"].get("GRBM_GUI_ACTIVE", 0.0)
        fetch = a["counters"].get("FETCH_SIZE", 0.0) * 1024
        write = b["counters"].get("WRITE_SIZE", 0.0) * 1024
        flop = busy * 1024.0
        grid = t.get("Grid_Size_X") or t.get("Grid_Size")
        # GEMMs of one grid differ by K: key by the MFMA work (FLOP, rounded to 1 %) as well
        key = (short(t["Kernel_Name"]), grid, round(flop / 1e9, 0) if flop > 1e9 else 0)
        g = groups.setdefault(key, dict(calls=0, us=0.0, flop=0.0, bytes=0.0, rbytes=0.0, wbytes=0.0, util=[], gui=0.0))
        g["calls"] += 1
        g["us"] += dur
        g["flop"] += flop
        g["bytes"] += 2 * fetch + write
        g["rbytes"] += 2 * fetch
        g["wbytes"] += write
        if gui > 0:
            g["util"].append(busy / (gui / 8.0 * 1024.0))
    print(f"# Roofline of one ViT-B/16 b256 training step (serial: bench.py --serial-wgrad), {n} dispatches, "
          f"{step_us / 1e3:.2f} ms of kernel time\n")
    print("Peaks: 2.5 PF bf16 dense MFMA, 8 TB/s HBM3E. FLOP from SQ_VALU_MFMA_BUSY_CYCLES x 1024; bytes = 2 x FETCH_SIZE + "
          "WRITE_SIZE (upper estimate of reads). `bound` = max(FLOP/peak, bytes/BW); `% of bound` = bound / measured.\n")
    print("| kernel | grid | calls | us/call | ms/step | GFLOP/call | TF/s | MFMA util | GB/call (r+w) | TB/s | bound | % of bound |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|---:|")
    rows = sorted(groups.items(), key=lambda kv: -kv[1]["us"])
    for (name, grid, _), g in rows:
        c = g["calls"]
        us = g["us"] / c
        if g["us"] < 20:
            continue
        fl = g["flop"] / c
        by = g["bytes"] / c
        tf = fl / (us * 1e-6) / 1e12
        bw = by / (us * 1e-6) / 1e12
        t_c, t_m = fl / PEAK_FLOPS * 1e6, by / PEAK_BW * 1e6
        bound = "MFMA" if t_c >= t_m else "HBM"
        pct = max(t_c, t_m) / us * 100
        util = sum(g["util"]) / len(g["util"]) * 100 if g["util"] else 0.0
        print(f"| `{name}` | {grid} | {c} | {us:.1f} | {g['us'] / 1e3:.3f} | {fl / 1e9:.1f} | {tf:.0f} | {util:.0f} % | "
              f"{g['rbytes'] / c / 1e9:.3f}+{g['wbytes'] / c / 1e9:.3f} | {bw:.2f} | {bound} | {pct:.0f} % |")


if __name__ == "__main__":
    main()
