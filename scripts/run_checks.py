#!/usr/bin/env python3
"""Run selected tests/kernel_checks.py checks by function name: python scripts/run_checks.py name[,name...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import kernel_checks as KC  # noqa: E402

names = sys.argv[1].split(",")
bad = 0
for fn in KC.all_checks():
    code = getattr(fn, "__code__", None)
    label = fn.__name__ if fn.__name__ != "<lambda>" else " ".join(code.co_names)
    if not any(n in label for n in names):
        continue
    torch.manual_seed(0)
    name, metrics, limits = fn()
    torch.cuda.synchronize()
    ok = KC.passed(metrics, limits)
    bad += not ok
    print(f"{'ok  ' if ok else 'FAIL'} {name}: {KC.fmt_metrics(metrics, limits)}", flush=True)
sys.exit(1 if bad else 0)
