#!/usr/bin/env python3
"""Attention forward / backward time at one model's shapes (default ViT-H/14 b128: N 257, H 16,
dh 80). usage: attn_shape_probe.py [B N H dh]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

B, N, H, dh = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (128, 257, 16, 80)
D = H * dh
ext = _ext.ext()
qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
scale = dh ** -0.5
o, lse = ext.attn_fwd(qkv, B, N, H, scale)
do = torch.randn_like(o)


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000


f = 4.0 * B * H * N * N * dh
tf = timed(lambda: ext.attn_fwd(qkv, B, N, H, scale))
tb = timed(lambda: ext.attn_bwd(do, qkv, o, lse, B, N, H, scale))
print(f"B{B} N{N} H{H} dh{dh}: fwd {tf:7.1f} us ({f / tf / 1e6:5.1f} TF)  "
      f"bwd {tb:7.1f} us ({2.5 * f / tb / 1e6:5.1f} TF)", flush=True)
