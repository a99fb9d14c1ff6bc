#!/usr/bin/env python3
"""Diagnostic: is the GEMM epilogue bound by chip-wide HBM write bandwidth when every CU stores at
once? Per-workgroup s_memtime stamps (tile 12, one 256x256 tile per workgroup) grouped by dispatch
round: a partial last round (few CUs storing) vs full rounds (all 256 CUs storing together)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

ext = _ext.ext()
T = 50432
seed = torch.tensor([5], dtype=torch.int64, device="cuda")
for (N, K, gelu, staged) in [(768, 768, False, 0), (768, 768, False, 1), (2304, 768, False, 0), (2304, 768, False, 1),
                             (3072, 768, True, 0), (3072, 768, True, 1)]:
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.empty(T, N, device="cuda", dtype=torch.bfloat16) if gelu else None
    nb = ((T + 255) // 256) * ((N + 255) // 256)
    dbg = torch.zeros(nb * 4, dtype=torch.int64, device="cuda")
    args = (x, True, w, True, y, T, N, K, 1 if gelu else 0, b, None, None, 0, aux, 0, 0, 0,
            seed if gelu else None, 3 << 32, 0.1 if gelu else 0.0, 0, 12)
    for _ in range(3):
        ext.gemm(*args, epi_staged=staged)
    torch.cuda.synchronize()
    ext.gemm(*args, dbg=dbg, epi_staged=staged)
    torch.cuda.synchronize()
    d = dbg.view(nb, 4).double().cpu()
    t0 = d[:, 0].min()
    order = torch.argsort(d[:, 0])
    pro, loop, epi = (d[:, 1] - d[:, 0]), (d[:, 2] - d[:, 1]), (d[:, 3] - d[:, 2])
    ncu = 256
    line = f"N{N} K{K} gelu{int(gelu)} staged{staged} blocks {nb}:"
    for r in range(min(2, (nb + ncu - 1) // ncu)):
        idx = order[r * ncu:(r + 1) * ncu]
        line += (f" | round {r} ({len(idx)} blk) pro {pro[idx].mean():.0f} loop {loop[idx].mean():.0f} "
                 f"epi {epi[idx].mean():.0f}")
    print(line, flush=True)
