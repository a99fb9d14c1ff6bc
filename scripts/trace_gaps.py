#!/usr/bin/env python3
"""GPU busy/idle analysis of a rocprofv3 kernel trace: union of kernel intervals vs wall time, the
largest idle gaps, and per-kernel totals within a window (the last `--steps` steps of the trace)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=0.0, help="analyse only the last N ms of the trace")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t_end = max(e for _, e, _ in ev)
    t0 = t_end - int(a.last_ms * 1e6) if a.last_ms else ev[0][0]
    ev = [x for x in ev if x[0] >= t0]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, n in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = cur_e - ev[0][0]
    print(f"window {wall / 1e6:.2f} ms: GPU busy {busy / 1e6:.2f} ms ({100 * busy / wall:.1f}%), idle {(wall - busy) / 1e6:.2f} ms "
          f"in {len(gaps)} gaps")
    for g, at, n in sorted(gaps, reverse=True)[:8]:
        print(f"  gap {g / 1e3:8.1f} us before {n[:90]}")


if __name__ == "__main__":
    main()
