import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# PVR_PKG_ROOT: a directory holding another build of the package (same-session A/B of a kernel
# variant against the same checks); it shadows the tree's own package
if os.environ.get("PVR_PKG_ROOT"):
    sys.path.insert(0, os.environ["PVR_PKG_ROOT"])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs on the gpurun box)")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Print every numerics check's measured errors next to its limits (tests/test_gpu_kernels.py)."""
    mod = sys.modules.get("tests.test_gpu_kernels")
    rows = getattr(mod, "MEASURED", None) if mod is not None else None
    if not rows:
        return
    from tests.kernel_checks import fmt_metrics, passed

    terminalreporter.section("kernel numerics: measured / limit")
    for name, metrics, limits in rows:
        terminalreporter.write_line(f"{'OK  ' if passed(metrics, limits) else 'FAIL'} {name}: {fmt_metrics(metrics, limits)}")
