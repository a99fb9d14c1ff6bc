#!/usr/bin/env python3
"""Diagnostic: per-workgroup s_memtime stamps of the GEMM kernels (prologue / main loop / epilogue)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

ext = _ext.ext()
T = 50432
for (N, K) in [(2304, 768), (768, 3072)]:
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    for tile, (BM, BN) in [(6, (256, 256)), (12, (256, 256))]:
        nb = ((T + BM - 1) // BM) * ((N + BN - 1) // BN)
        dbg = torch.zeros(nb * 4, dtype=torch.int64, device="cuda")
        args = (x, True, w, True, y, T, N, K, 0, b, None, None, 0, None, 0, 0, 0, None, 0, 0.0, 0, tile)
        for _ in range(3):
            ext.gemm(*args)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ext.gemm(*args, dbg=dbg)
        e.record()
        torch.cuda.synchronize()
        d = dbg.view(nb, 4).double().cpu()
        pro, loop, epi = (d[:, 1] - d[:, 0]), (d[:, 2] - d[:, 1]), (d[:, 3] - d[:, 2])
        t0 = d[:, 0].min()
        span = (d[:, 3].max() - t0)
        print(f"N{N} K{K} tile{tile} ({BM}x{BN}) blocks {nb}: wall {s.elapsed_time(e):.3f} ms | per-block cycles(memtime) "
              f"prologue {pro.mean():.0f} loop {loop.mean():.0f} (min {loop.min():.0f} max {loop.max():.0f}) "
              f"epilogue {epi.mean():.0f} | total span {span:.0f} | blocks/span-start-quartiles "
              f"{[float(q) for q in torch.quantile(d[:, 0] - t0, torch.tensor([0.25, 0.5, 0.75], dtype=torch.float64))]}",
              flush=True)
