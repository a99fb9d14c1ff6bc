#!/usr/bin/env python3
"""Tile-config sweep of the ViT-B/16 b256 forward / dgrad GEMMs with their in-step epilogues
(ms and TFLOP/s per config; unsupported layout / config pairs are skipped)."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402
from bench_kernels import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    T, D, M = 256 * 197, 768, 3072
    x = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
    h = torch.randn(T, M, device=dev, dtype=torch.bfloat16)
    r = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
    wo = (torch.randn(D, D, device=dev) * 0.02).to(torch.bfloat16)
    wq = (torch.randn(3 * D, D, device=dev) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(D, M, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(D, device=dev)
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    dq = torch.randn(T, 3 * D, device=dev, dtype=torch.bfloat16)
    wot, wqt = wo.t().contiguous(), wq.t().contiguous()
    cases = [
        ("out fwd  bias+resid", 2.0 * T * D * D, lambda: G.linear_fwd(x, wo, b, resid=r)),
        ("out dgrad (wT)", 2.0 * T * D * D, lambda: G.linear_dgrad(r, wo, wt=wot)),
        ("qkv dgrad (wT)", 2.0 * T * D * 3 * D, lambda: G.linear_dgrad(dq, wq, wt=wqt)),
        ("fc2 fwd  bias+drop+resid", 2.0 * T * D * M, lambda: G.linear_fwd(h, w2, b, resid=r, drop=(seed, 4 << 32, 0.1))),
    ]
    for name, fl, fn in cases:
        res = []
        for t in [None] + list(range(0, 14)):
            G._FORCE_TILE = None if t is None else str(t)
            try:
                ms = timeit(fn)
            except Exception:  # noqa: BLE001 - unsupported config for this layout
                continue
            finally:
                G._FORCE_TILE = None
            res.append((ms, "default" if t is None else f"tile{t}"))
        line = " ".join(f"{n}={ms:.3f}({fl / ms / 1e9:.0f}TF)" for ms, n in res)
        print(f"{name}: {line}", flush=True)


if __name__ == "__main__":
    main()
