"""Run the attention kernels at ViT-B/16 b256 shapes a few times (for rocprofv3 counter collection).

usage: attn_probe.py [fwd|bwd|both]   (PVR_ATTN_BWD_PIPE=0 selects the two-kernel backward)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
ext = _ext.ext()
# PVR_PROBE_SHAPE="B,N,H,dh" (default ViT-B/16 b256)
B, N, H, dh = (int(v) for v in os.environ.get("PVR_PROBE_SHAPE", "256,197,12,64").split(","))
D = H * dh
qkv = torch.randn(B * N, 3 * D, device="cuda", dtype=torch.bfloat16)
o, lse = ext.attn_fwd(qkv, B, N, H, dh ** -0.5)
do = torch.randn_like(o)
for _ in range(3):
    if which in ("fwd", "both"):
        ext.attn_fwd(qkv, B, N, H, dh ** -0.5)
    if which in ("bwd", "both"):
        # with the in-step bias partials when the pipelined backward serves the shape
        part = (torch.empty(B * H, (N + 31) // 32, 192, device="cuda", dtype=torch.float32)
                if ext.attn_bwd_pipe_path(B, N, H, D) else None)
        ext.attn_bwd(do, qkv, o, lse, B, N, H, dh ** -0.5, None, part)
torch.cuda.synchronize()
print("ok")
