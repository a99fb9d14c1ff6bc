"""Per-part (dQ / dK / dV) error of the attention backward vs the fp32 reference, per shape."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("PVR_PKG_ROOT"):  # an alternative build of the package (A/B), e.g. ab_safe/
    sys.path.insert(0, os.path.join(ROOT, os.environ["PVR_PKG_ROOT"]))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from tests.kernel_checks import _attn_ref  # noqa: E402

ext = _ext.ext()
print("package:", _ext.__file__)
shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(1, 197, 1), (2, 197, 3), (1, 256, 1), (1, 224, 1), (4, 197, 2)]
for (B, N, H) in shapes:
    torch.manual_seed(0)
    D = H * 64
    qkv = (torch.randn(B * N, 3 * D, device="cuda")).bfloat16()
    o, lse = ext.attn_fwd(qkv, B, N, H, 0.125)
    do = torch.randn(B * N, D, device="cuda").bfloat16()
    dqkv = ext.attn_bwd(do, qkv, o, lse, B, N, H, 0.125, None).float()
    qr = qkv.float().requires_grad_(True)
    oref, _ = _attn_ref(qr, B, N, H)
    oref.backward(do.float())
    g = qr.grad
    msg = []
    for i, nm in enumerate("QKV"):
        a, r = dqkv[:, i * D:(i + 1) * D], g[:, i * D:(i + 1) * D]
        e = (a - r).abs().max().item() / max(1.0, r.abs().max().item())
        rows = ((a - r).abs().amax(1) > 0.05 * max(1.0, r.abs().max().item())).nonzero().flatten().tolist()
        cols = ((a - r).abs().amax(0) > 0.05 * max(1.0, r.abs().max().item())).nonzero().flatten().tolist()
        msg.append(f"d{nm} err {e:.3e} badrows {rows[:6]}..{len(rows)} badcols {cols[:6]}..{len(cols)}")
    print(f"B{B} N{N} H{H}: " + " | ".join(msg), flush=True)
