"""scripts/fp8_study_stats.py: the seed-study statistics (per-checkpoint mean +- std, paired
differences by seed, paired t-test, within-one-bf16-sigma flag) from '[ckpt]' log lines. CPU only."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(seed, variant, losses):
    return "[ckpt] " + json.dumps({"seed": seed, "variant": variant, "window": 20, "loss": losses, "train_s": 1.0})


def test_fp8_study_stats_paired_test(tmp_path):
    scipy = pytest.importorskip("scipy.stats")
    bf = {0: 1.00, 1: 1.20, 2: 0.90, 3: 1.10, 4: 1.05}
    lines = []
    for s, v in bf.items():
        lines.append(_line(s, "fused", {"200": v, "400": v / 2}))
        lines.append(_line(s, "fused_fp8", {"200": v + 0.01 * (s + 1), "400": v / 2}))  # small, consistent gap at 200
        lines.append(_line(s, "fused_fp8w", {"200": v + 0.5, "400": v / 2 + 0.001}))     # large gap at 200
    log = tmp_path / "study.log"
    log.write_text("noise line\n" + "\n".join(lines) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "fp8_study_stats.py"), str(log)],
                         capture_output=True, text=True, check=True).stdout
    summary = json.loads(out.strip().splitlines()[-1])
    assert summary["seeds"] == [0, 1, 2, 3, 4] and summary["steps"] == [200, 400]
    rows = {(r["step"], r["variant"]): r for r in summary["rows"]}
    r = rows[(200, "fused_fp8")]
    x = [bf[s] + 0.01 * (s + 1) for s in bf]
    assert r["p_paired"] == pytest.approx(float(scipy.ttest_rel(x, list(bf.values())).pvalue))
    assert r["diff_mean"] == pytest.approx(0.03)
    assert r["within_1sd"]
    assert not rows[(200, "fused_fp8w")]["within_1sd"]
    assert rows[(400, "fused_fp8")]["diff_mean"] == pytest.approx(0.0)


def test_fp8_study_stats_e4m3_vs_e5m2(tmp_path):
    """With both fp8-wgrad arms present (e5m2: fused_fp8w, e4m3: fused_fp8w4), the script also pairs
    e4m3 against e5m2 by seed."""
    scipy = pytest.importorskip("scipy.stats")
    bf = {0: 1.00, 1: 1.20, 2: 0.90, 3: 1.10}
    lines = []
    for s, v in bf.items():
        lines.append(_line(s, "fused", {"200": v}))
        lines.append(_line(s, "fused_fp8w", {"200": v + 0.2}))
        lines.append(_line(s, "fused_fp8w4", {"200": v + 0.1 - 0.01 * s}))
    log = tmp_path / "study.log"
    log.write_text("\n".join(lines) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "fp8_study_stats.py"), str(log)],
                         capture_output=True, text=True, check=True).stdout
    summary = json.loads(out.strip().splitlines()[-1])
    assert {r["variant"] for r in summary["rows"]} == {"fused_fp8w", "fused_fp8w4"}
    (row,) = summary["e4m3_vs_e5m2"]
    a4 = [v + 0.1 - 0.01 * s for s, v in bf.items()]
    a5 = [v + 0.2 for v in bf.values()]
    assert row["step"] == 200 and row["diff_mean"] == pytest.approx(sum(a - b for a, b in zip(a4, a5)) / 4)
    assert row["p_paired"] == pytest.approx(float(scipy.ttest_rel(a4, a5).pvalue))
    assert "| e4m3 grads | e5m2 grads |" in out
