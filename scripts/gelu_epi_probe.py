#!/usr/bin/env python3
"""fc1 forward (bias + GELU + dropout + saved derivative) at ViT-B/16 b256 with one experiment
build of the extension: PVR_EXP=0 normal, 1 no aux store, 2 no GELU math. usage: gelu_epi_probe.py <tree>"""
import sys

import torch

sys.path.insert(0, sys.argv[1])
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402

T, D, M = 50432, 768, 3072
x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
w = (torch.randn(M, D, device="cuda") * 0.03).to(torch.bfloat16)
b = torch.randn(M, device="cuda")
u = torch.empty(T, M, dtype=torch.bfloat16, device="cuda")
seed = torch.tensor([5], dtype=torch.int64, device="cuda")
for tile in ("13", "12"):
    G._FORCE_TILE = tile
    fn = lambda: G.linear_fwd(x, w, b, gelu_aux=u, drop=(seed, 3 << 32, 0.1))  # noqa: E731
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{sys.argv[1]} tile{tile}: fc1 fwd GELU {s.elapsed_time(e) / 20 * 1000:.1f} us", flush=True)
