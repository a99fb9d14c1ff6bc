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
        for v in ("fused_fp8", "fused_fp8w"):
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
    print(json.dumps(out))


if __name__ == "__main__":
    main()
