"""GPU numerics tests: every HIP kernel vs a PyTorch fp32 reference (see tests/kernel_checks.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from tests import kernel_checks as KC

    CHECKS = KC.all_checks()
else:  # pragma: no cover
    CHECKS = []


@pytest.mark.parametrize("idx", range(len(CHECKS)) if CHECKS else [0])
def test_kernel_numerics(idx):
    if not CHECKS:
        pytest.skip("no GPU")
    from pytorch_vit_paper_replication_amd import _ext

    assert _ext.available(), "HIP extension must be loaded on a GPU box"
    torch.manual_seed(idx)
    name, err, tol = CHECKS[idx]()
    torch.cuda.synchronize()
    assert err <= tol, f"{name}: err {err:.3e} > tol {tol:.1e}"
