"""fp8 configuration on the CPU: ``ViT.enable_fp8(grad_fmt=...)`` chooses the gradients' fp8 format
(e4m3 default since round 6, e5m2), a format change starts a fresh scaling state, the resume state records the
format and refuses a mismatch, and bench.py parses ``--fp8-grad``. The kernels that take the format
are checked on the GPU (tests/kernel_checks.py, ``fmt=0`` rows and ``check_vit_fp8_grad_formats``)."""
import pytest
import torch

from pytorch_vit_paper_replication_amd.models import ViT
from pytorch_vit_paper_replication_amd.ops import fp8 as F8

from .test_bench_cli import _bench


def _small():
    return ViT(image_size=32, patch_size=16, num_transformer_layer=2, num_heads=2, embedding_dim=128, mlp_size=256,
               num_classes=10)


def test_enable_fp8_grad_fmt_config():
    m = _small()
    m.enable_fp8()
    assert m._fp8_cfg[4] == "e4m3"  # the default since round 6
    st = m._fp8_state(torch.device("cpu"), 1024)
    assert st is not None and st.grad.fmt == F8.E4M3 and st.act.fmt == F8.E4M3
    assert float(st.grad.fmax[0]) == 448.0
    m.enable_fp8(dgrad=False)  # a dgrad switch keeps the scaling state
    assert m._fp8_state(torch.device("cpu"), 1024) is st
    m.enable_fp8(grad_fmt="e5m2")  # a format switch starts a fresh one
    st5 = m._fp8_state(torch.device("cpu"), 1024)
    assert st5 is not st and st5.grad.fmt == F8.E5M2 and float(st5.grad.fmax[0]) == 57344.0
    with pytest.raises(ValueError):
        m.enable_fp8(grad_fmt="e3m4")


def test_fp8_state_records_grad_fmt():
    st4 = F8.Fp8State(2, "cpu", grad_fmt=F8.E4M3)
    sd = st4.state_dict()
    assert int(sd["grad_fmt"]) == F8.E4M3
    F8.Fp8State(2, "cpu", grad_fmt=F8.E4M3).load_state_dict(sd)
    with pytest.raises(ValueError):
        F8.Fp8State(2, "cpu", grad_fmt=F8.E5M2).load_state_dict(sd)  # e5m2 model, e4m3 checkpoint
    old = {k: v for k, v in F8.Fp8State(2, "cpu", grad_fmt=F8.E5M2).state_dict().items() if k != "grad_fmt"}
    F8.Fp8State(2, "cpu").load_state_dict(old)  # checkpoints from before the format field (e5m2) still load
    with pytest.raises(ValueError):
        F8.Fp8State(2, "cpu", grad_fmt=7)


def test_bench_fp8_grad_flag():
    import sys

    bench = _bench()
    old = sys.argv
    try:
        sys.argv = ["bench.py", "--model", "vit_h14", "--dtype", "fp8", "--fp8-grad", "e4m3"]
        assert bench.parse().fp8_grad == "e4m3"
        sys.argv = ["bench.py", "--dtype", "fp8", "--fp8-grad", "e5m2"]
        assert bench.parse().fp8_grad == "e5m2"
        sys.argv = ["bench.py"]
        assert bench.parse().fp8_grad == "e4m3"
    finally:
        sys.argv = old
