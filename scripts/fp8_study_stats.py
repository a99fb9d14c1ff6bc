#!/usr/bin/env python3
"""Statistics of an fp8 seed study (scripts/convergence_check.py --fp8-study --checkpoints ...): reads
the '[ckpt] {...}' JSON lines of one or more logs and prints, per checkpoint step and fp8 variant, the
mean +- std of the windowed training loss over seeds next to bf16's, the paired difference (same
init and batch order per seed) with a paired t-test, and whether the variant's mean lies within one
bf16 standard deviation.

  python scripts/fp8_study_stats.py profiles/r6/fp8_study/*.log
"""
import json
import sys
from collections import defaultdict

from scipy import stats


def main():
    runs = defaultdict(dict)  # variant -> seed -> {step: loss}
    for path in sys.argv[1:]:
        for line in open(path):
            if line.startswith("[ckpt] "):
                d = json.loads(line[7:])
                runs[d["variant"]][d["seed"]] = {int(k): v for k, v in d["loss"].items()}
    base = runs.get("fused", {})
    seeds = sorted(base)
    steps = sorted({s for r in base.values() for s in r})
    out = {"seeds": seeds, "steps": steps, "rows": []}
    print(f"# fp8 seed study: {len(seeds)} seeds {seeds}; windowed training loss at each step (mean +- std over seeds)")
    print("| step | variant | loss | bf16 loss | paired diff (variant - bf16) | paired t-test p | within 1 bf16 sd |")
    print("|---:|---|---:|---:|---:|---:|---|")
    for st in steps:
        b = [base[s][st] for s in seeds]
        bm, bs = sum(b) / len(b), stats.tstd(b) if len(b) > 1 else 0.0
        for v in [v for v in ("fused_fp8", "fused_fp8w", "fused_fp8w4") if v in runs] + sorted(
                v for v in runs if v not in ("fused", "fused_fp8", "fused_fp8w", "fused_fp8w4")):
            if v not in runs:
                continue
            sv = [s for s in seeds if s in runs[v] and st in runs[v][s]]
            x = [runs[v][s][st] for s in sv]
            bb = [base[s][st] for s in sv]
            d = [a - c for a, c in zip(x, bb)]
            m, sd = sum(x) / len(x), stats.tstd(x) if len(x) > 1 else 0.0
            dm, dsd = sum(d) / len(d), stats.tstd(d) if len(d) > 1 else 0.0
            p = float(stats.ttest_rel(x, bb).pvalue) if len(x) > 1 else float("nan")
            within = abs(m - bm) <= bs
            out["rows"].append({"step": st, "variant": v, "mean": m, "std": sd, "bf16_mean": bm, "bf16_std": bs,
                                "diff_mean": dm, "diff_std": dsd, "p_paired": p, "within_1sd": bool(within)})
            print(f"| {st} | {v} | {m:.4f} +- {sd:.4f} | {bm:.4f} +- {bs:.4f} | {dm:+.4f} +- {dsd:.4f} | {p:.3f} | {'yes' if within else 'no'} |")
    if "fused_fp8w" in runs and "fused_fp8w4" in runs:  # e4m3 vs e5m2 gradients, paired by seed
        print("\n| step | e4m3 grads | e5m2 grads | paired diff (e4m3 - e5m2) | paired t-test p |")
        print("|---:|---:|---:|---:|---:|")
        for st in steps:
            sv = [s for s in seeds if st in runs["fused_fp8w"].get(s, {}) and st in runs["fused_fp8w4"].get(s, {})]
            if len(sv) < 2:
                continue
            a4 = [runs["fused_fp8w4"][s][st] for s in sv]
            a5 = [runs["fused_fp8w"][s][st] for s in sv]
            d = [x - y for x, y in zip(a4, a5)]
            p = float(stats.ttest_rel(a4, a5).pvalue)
            out.setdefault("e4m3_vs_e5m2", []).append({"step": st, "e4m3": sum(a4) / len(a4), "e5m2": sum(a5) / len(a5),
                                                       "diff_mean": sum(d) / len(d), "diff_std": stats.tstd(d), "p_paired": p})
            print(f"| {st} | {sum(a4) / len(a4):.4f} +- {stats.tstd(a4):.4f} | {sum(a5) / len(a5):.4f} +- {stats.tstd(a5):.4f} | "
                  f"{sum(d) / len(d):+.4f} +- {stats.tstd(d):.4f} | {p:.3f} |")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
