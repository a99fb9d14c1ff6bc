"""GPU numerics tests: every HIP kernel vs a PyTorch fp32 reference (see tests/kernel_checks.py).

Each check's measured errors are recorded and printed in the pytest terminal summary (``conftest.py``),
so the log of ``pytest -m gpu`` shows every value next to its limit."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from tests import kernel_checks as KC

    CHECKS = KC.all_checks()
else:  # pragma: no cover
    CHECKS = []

MEASURED = []  # (name, metrics, limits) of every check run in this session (conftest prints them)


@pytest.mark.parametrize("idx", range(len(CHECKS)) if CHECKS else [0])
def test_kernel_numerics(idx):
    if not CHECKS:
        pytest.skip("no GPU")
    from pytorch_vit_paper_replication_amd import _ext

    assert _ext.available(), "HIP extension must be loaded on a GPU box"
    torch.manual_seed(idx)
    name, metrics, limits = CHECKS[idx]()
    torch.cuda.synchronize()
    MEASURED.append((name, metrics, limits))
    assert KC.passed(metrics, limits), f"{name}: {KC.fmt_metrics(metrics, limits)}"
