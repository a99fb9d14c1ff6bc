#!/usr/bin/env python3
"""One GEMM kind in a loop, for PMC counter passes (rocprofv3 --pmc ... -- python3 scripts/gemm_pmc_probe.py):
the ViT-B/16 b256 qkv weight gradient (mn-contiguous operands, split-K partials, tile 12/14) and the
qkv forward (k-contiguous, persistent ping-pong) at the same FLOP count.

  python scripts/gemm_pmc_probe.py --kind wgrad --iters 20
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=["wgrad", "fwd", "both"], default="both")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    T, D = 50432, 768
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    d3 = torch.randn(T, 3 * D, device="cuda").to(torch.bfloat16)
    w = (torch.randn(3 * D, D, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(3 * D, device="cuda")
    ws = torch.zeros(3 * D, D, device="cuda")
    out = torch.empty(T, 3 * D, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.iters):
        if a.kind in ("wgrad", "both"):
            G.linear_wgrad(d3, x, ws)
        if a.kind in ("fwd", "both"):
            G.linear_fwd(x, w, b, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        if a.kind in ("wgrad", "both"):
            G.linear_wgrad(d3, x, ws)
    e.record()
    torch.cuda.synchronize()
    fl = 2.0 * T * 3 * D * D
    t = s.elapsed_time(e) / a.iters
    print(f"qkv wgrad {t:.4f} ms {fl / t / 1e9:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
