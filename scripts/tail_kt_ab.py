#!/usr/bin/env python3
"""A/B of the split-K tail's smallest part (ext.set_gemm_tail_min_kt) on the short-K GEMMs of
ViT-H/14 fp8 (K = 1280: 10 K-tiles) and ViT-B/16 bf16 (K = 768: 12 K-tiles), same process,
alternating order per round; median ms.

  python scripts/tail_kt_ab.py [--rounds 4] [--kts 12,6,4,3]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import fp8 as F8  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20, warmup=4):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


class Meta:
    def __init__(self, dev, fmt):
        self.qscale = torch.ones(1, device=dev)
        self.amax = torch.zeros(1, dtype=torch.int32, device=dev)
        self.dscale = torch.ones(1, device=dev)
        self.fmt = fmt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--kts", default="12,6,4,3")
    a = ap.parse_args()
    kts = [int(k) for k in a.kts.split(",")]
    dev = "cuda"
    ext = _ext.ext()
    torch.manual_seed(0)
    s = torch.ones(1, device=dev)
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    drop = (seed, 3 << 32, 0.1)
    cases = []
    # ViT-H/14 fp8, batch 256
    D, M, T = 1280, 5120, 256 * 257
    f8 = lambda *shape: (torch.randn(*shape, device=dev) * 0.5).to(torch.float8_e4m3fn).view(torch.uint8)  # noqa: E731
    x8, h8 = f8(T, D), f8(T, M)
    g8 = (torch.randn(T, D, device=dev)).to(torch.float8_e5m2).view(torch.uint8)
    w = {"qkv": f8(3 * D, D), "out": f8(D, D), "fc1": f8(M, D), "fc2t": f8(M, D), "outt": f8(D, D)}
    b = {"qkv": torch.randn(3 * D, device=dev), "out": torch.randn(D, device=dev), "fc1": torch.randn(M, device=dev)}
    resid = torch.randn(T, D, device=dev).to(torch.bfloat16)
    aux = torch.empty(T, M, dtype=torch.bfloat16, device=dev)
    colsum = torch.zeros(M, device=dev)
    m4, m5 = Meta(dev, 0), Meta(dev, 1)
    cases += [
        ("h14 qkv fwd (3855 tiles)", lambda: F8.linear_fwd_fp8(x8, s, w["qkv"], s, b["qkv"])),
        ("h14 out fwd +resid (1285)", lambda: F8.linear_fwd_fp8(x8, s, w["out"], s, b["out"], resid=resid, drop=drop)),
        ("h14 fc1 fwd GELU step (5140)", lambda: F8.linear_fwd_fp8(x8, s, w["fc1"], s, b["fc1"], gelu_aux=aux, drop=drop,
                                                                  quant=(m4, 0), skip_out=True)),
        ("h14 out dgrad (1285)", lambda: F8.linear_dgrad_fp8(g8, s, w["outt"], s)),
        ("h14 fc2 dgrad dGELU step (5140)", lambda: F8.linear_dgrad_fp8(g8, s, w["fc2t"], s, dgelu_aux=aux, colsum=colsum,
                                                                       quant=(m5, 0), skip_out=True)),
    ]
    # ViT-B/16 bf16, batch 256
    Db, Tb = 768, 256 * 197
    xb = torch.randn(Tb, Db, device=dev).to(torch.bfloat16)
    wo = (torch.randn(Db, Db, device=dev) * 0.02).to(torch.bfloat16)
    wq = (torch.randn(3 * Db, Db, device=dev) * 0.02).to(torch.bfloat16)
    rb = torch.randn(Tb, Db, device=dev).to(torch.bfloat16)
    cases += [
        ("b16 qkv fwd (591 tiles)", lambda: G.linear_fwd(xb, wq)),
        ("b16 out fwd +resid (197)", lambda: G.linear_fwd(xb, wo, resid=rb, drop=drop)),
        ("b16 out dgrad (197)", lambda: G.linear_dgrad(xb, wo, wt=wo.t().contiguous())),
    ]
    res = {}
    for rnd in range(a.rounds):
        order = kts if rnd % 2 == 0 else kts[::-1]
        for name, fn in cases:
            for kt in order:
                ext.set_gemm_tail_min_kt(kt)
                res.setdefault((name, kt), []).append(timeit(fn))
    ext.set_gemm_tail_min_kt(12)
    print("# split-tail smallest part (K-tiles): " + " | ".join(f"min {k}" for k in kts) + "  (median ms)", flush=True)
    for name, _ in cases:
        print(f"{name:34s} " + " | ".join(f"{statistics.median(res[(name, k)]):7.4f}" for k in kts), flush=True)


if __name__ == "__main__":
    main()
