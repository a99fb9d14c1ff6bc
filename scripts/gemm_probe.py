#!/usr/bin/env python3
"""Run one GEMM shape through our kernel (given tile configs) and hipBLASLt, a few times each,
for rocprofv3 PMC collection (one dispatch row per kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402

T, N, K = 50432, int(os.environ.get("PN", 2304)), int(os.environ.get("PK", 768))
tiles = [int(t) for t in os.environ.get("PTILES", "0,3").split(",")]
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
b = torch.randn(N, device="cuda")
for t in tiles:
    G.FORCE_TILE = t
    for _ in range(3):
        G.linear_fwd(x, w, b)
for _ in range(3):
    torch.matmul(x, w.t())
torch.cuda.synchronize()
print("done")
