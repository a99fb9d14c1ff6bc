#!/usr/bin/env python3
"""Attention forward at the ViT-H/14 b256 and ViT-L/16@384 b128 shapes with and without the e4m3 copy
of O (the fp8 step writes it for the out-proj GEMM), O stored through LDS (default) or straight from
the registers (ext.set_attn_fwd_direct), alternating; median ms.

  python scripts/attn_q8_probe.py
"""
from __future__ import annotations

import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402


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


def main():
    ext = _ext.ext()
    dev = "cuda"
    for name, B, N, H, D in (("h14", 256, 257, 16, 1280), ("l16_384", 128, 577, 16, 1024)):
        qkv = (torch.randn(B * N, 3 * D, device=dev) * 0.5).to(torch.bfloat16)
        q8 = torch.empty(B * N, D, dtype=torch.uint8, device=dev)
        qs = torch.ones(1, device=dev)
        am = torch.zeros(1, dtype=torch.int32, device=dev)
        sc = (D // H) ** -0.5
        res = {}
        variants = [(cp, st) for cp in ("plain", "q8") for st in ("staged", "direct")]
        for rnd in range(5):
            for v in (variants if rnd % 2 == 0 else variants[::-1]):
                ext.set_attn_fwd_direct(v[1] == "direct")
                if v[0] == "plain":
                    fn = lambda: ext.attn_fwd(qkv, B, N, H, sc)  # noqa: E731
                else:
                    fn = lambda: ext.attn_fwd(qkv, B, N, H, sc, None, 0, 0.0, q8, qs, am)  # noqa: E731
                res.setdefault(v, []).append(timeit(fn))
        ext.set_attn_fwd_direct(False)
        print(f"attn fwd {name:8s} B{B} N{N} H{H}: " + " | ".join(
            f"{cp} {st} {statistics.median(res[(cp, st)]):.4f} ms" for cp, st in variants), flush=True)


if __name__ == "__main__":
    main()
