#!/usr/bin/env python3
"""Cost of each part of the fc1 forward epilogue (GELU, derivative store, dropout, fp8 copy) and of
the dGELU dgrad epilogue: the same GEMM timed with the epilogue features switched on one by one.

  python scripts/fc1_epi_probe.py [--model h14|b16]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import fp8 as F8  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20, warmup=5):
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


class Meta:  # one delayed-scaling slot
    def __init__(self, dev, fmt):
        self.qscale = torch.ones(1, device=dev)
        self.amax = torch.zeros(1, dtype=torch.int32, device=dev)
        self.dscale = torch.ones(1, device=dev)
        self.fmt = fmt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="h14")
    ap.add_argument("--persistent", type=int, default=None, help="ext.set_fp8_persistent mode (A/B)")
    a = ap.parse_args()
    if a.persistent is not None:
        _ext.ext().set_fp8_persistent(a.persistent)
    dev = "cuda"
    D, M, B = (1280, 5120, 256) if a.model == "h14" else (768, 3072, 256)
    T = B * (257 if a.model == "h14" else 197)
    torch.manual_seed(0)
    x = torch.randn(T, D, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(M, D, device=dev) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(D, M, device=dev) * 0.02).to(torch.bfloat16)
    w2t = w2.t().contiguous()  # W2^T rows for the dgrad
    b1 = torch.randn(M, device=dev) * 0.1
    aux = torch.empty(T, M, dtype=torch.bfloat16, device=dev)
    dz = (torch.randn(T, D, device=dev) * 1e-2).to(torch.bfloat16)
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    drop = (seed, 3 << 32, 0.1)
    fl = 2.0 * T * M * D
    rows = []
    if a.model == "h14":
        x8 = (x.float() * 8).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
        w18 = (w1.float() * 64).to(torch.float8_e4m3fn).view(torch.uint8)
        w2t8 = (w2t.float() * 64).to(torch.float8_e4m3fn).view(torch.uint8)
        dz8 = (dz.float() * 1000).to(torch.float8_e5m2).view(torch.uint8)
        s = torch.ones(1, device=dev)
        m4, m5 = Meta(dev, 0), Meta(dev, 1)
        colsum = torch.zeros(M, device=dev)
        rows += [
            ("fwd bias only (bf16 out)", lambda: F8.linear_fwd_fp8(x8, s, w18, s, b1)),
            ("fwd GELU + aux", lambda: F8.linear_fwd_fp8(x8, s, w18, s, b1, gelu_aux=aux)),
            ("fwd GELU + aux + drop", lambda: F8.linear_fwd_fp8(x8, s, w18, s, b1, gelu_aux=aux, drop=drop)),
            ("fwd GELU + aux + drop + e4m3 (bf16 too)", lambda: F8.linear_fwd_fp8(x8, s, w18, s, b1, gelu_aux=aux, drop=drop,
                                                                                quant=(m4, 0))),
            ("fwd GELU + aux + drop + e4m3 only (step)", lambda: F8.linear_fwd_fp8(x8, s, w18, s, b1, gelu_aux=aux, drop=drop,
                                                                                 quant=(m4, 0), skip_out=True)),
            ("dgrad plain (K = 1280 -> 5120)", lambda: F8.linear_dgrad_fp8(dz8, s, w2t8, s)),
            ("dgrad dGELU + colsum + e5m2 only (step)", lambda: F8.linear_dgrad_fp8(dz8, s, w2t8, s, dgelu_aux=aux, colsum=colsum,
                                                                                  quant=(m5, 0), skip_out=True)),
        ]
    else:
        colsum = torch.zeros(M, device=dev)
        rows += [
            ("fwd bias only", lambda: G.linear_fwd(x, w1, b1)),
            ("fwd GELU + aux", lambda: G.linear_fwd(x, w1, b1, gelu_aux=aux, gelu=True)),
            ("fwd GELU + aux + drop (step)", lambda: G.linear_fwd(x, w1, b1, gelu_aux=aux, gelu=True, drop=drop)),
            ("dgrad plain", lambda: G.linear_dgrad(dz, w2, wt=w2t)),
            ("dgrad dGELU + colsum (step)", lambda: G.linear_dgrad(dz, w2, wt=w2t, dgelu_aux=aux, colsum=colsum)),
        ]
    for name, fn in rows:
        t = min(timeit(fn) for _ in range(3))
        print(f"{a.model} {name:44s} {t:7.3f} ms {fl / t / 1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
