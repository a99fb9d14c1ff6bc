#!/usr/bin/env python3
"""Every GEMM tile config on the N = 768 GEMMs of ViT-B/16 b256 (591 256x256 tiles = 2.3 waves on
256 CUs): out-proj / fc2 forward with their epilogues and the k-contiguous (W^T) dgrads."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402

dev = "cuda"
T, D, M = 50432, 768, 3072
bf = lambda *s, sc=1.0: (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)  # noqa: E731
o, x, h = bf(T, D), bf(T, D), bf(T, M)
wo, w2 = bf(D, D, sc=0.03), bf(D, M, sc=0.02)
bo, b2 = torch.randn(D, device=dev), torch.randn(D, device=dev)
dq, w1 = bf(T, 3 * D), bf(M, D, sc=0.03)
wq = bf(3 * D, D, sc=0.03)
seed = torch.tensor([5], dtype=torch.int64, device=dev)
cases = {
    "out fwd bias+resid      K768 ": (2.0 * T * D * D, lambda: G.linear_fwd(o, wo, bo, resid=x)),
    "fc2 fwd bias+drop+resid K3072": (2.0 * T * D * M, lambda: G.linear_fwd(h, w2, b2, resid=x, drop=(seed, 9 << 32, 0.1))),
    "qkv dgrad (wT)          K2304": (2.0 * T * D * 3 * D, lambda: G.linear_dgrad(dq, wq, wt=wq.t().contiguous())),
    "fc1 dgrad (wT)          K3072": (2.0 * T * D * M, lambda: G.linear_dgrad(h, w1, wt=w1.t().contiguous())),
}


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for name, (fl, fn) in cases.items():
    for tile in (12, 13, 6, 9, 10, 11):
        G._FORCE_TILE = str(tile)
        try:
            ms = timed(fn)
            print(f"{name} tile{tile:2d} {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF", flush=True)
        except Exception as ex:  # unsupported layout for this config
            print(f"{name} tile{tile:2d} n/a ({str(ex)[:60]})", flush=True)
    G._FORCE_TILE = None
