#!/usr/bin/env python3
"""Deferred-epilogue GELU GEMM (gemm_ppd_kernel) vs the one-pass persistent kernel (tile 13):
bit-equality of output and saved derivative (same fp32 accumulation order, same epilogue math), then
alternating timings at the fc1 shapes.

  python scripts/gemm_deferred_ab.py
"""
from __future__ import annotations

import os
import statistics
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

SHAPES = [  # (name, M, N, K): fc1 of ViT-B/16 b256, ViT-L/16-384 b128, ViT-H/14 b256; odd tails
    ("b16 fc1", 50432, 3072, 768), ("l16 fc1", 73856, 4096, 1024), ("h14 fc1", 65792, 5120, 1280),
    ("tail M", 5000, 3072, 768), ("tail N", 9000, 1000, 256), ("short K", 6000, 768, 128)]


def run(ext, x, w, b, out, aux, seed, M, N, K, p):
    ext.gemm(x, True, w, True, out, M, N, K, 1, b, None, None, 0, aux, 0, 0, 0, seed, 3 << 32, p, 0, 13, tail_limit=-1)


def main():
    ext = _ext.ext()
    seed = torch.tensor([12345], dtype=torch.int64, device="cuda")
    ok = True
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda") * 0.1
        res = {}
        for d in (0, 1):
            ext.set_gemm_deferred(d)
            for p in (0.0, 0.1):
                out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
                aux = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
                run(ext, x, w, b, out, aux, seed, M, N, K, p)
                torch.cuda.synchronize()
                res[(d, p)] = (out, aux)
        for p in (0.0, 0.1):
            o0, a0 = res[(0, p)]
            o1, a1 = res[(1, p)]
            eq_o = torch.equal(o0.view(torch.int16), o1.view(torch.int16))
            eq_a = torch.equal(a0.view(torch.int16), a1.view(torch.int16))
            nan = bool(torch.isnan(o1).any() or torch.isnan(a1).any())
            ok &= eq_o and eq_a and not nan
            print(f"{name:8s} M{M} N{N} K{K} p{p}: out bit-equal {eq_o}, aux bit-equal {eq_a}, unwritten {nan}", flush=True)
        del res
    ext.set_gemm_deferred(0)
    if not ok:
        print("MISMATCH", flush=True)
        sys.exit(1)
    if os.environ.get("PPD_CHECK_ONLY"):
        return
    # timing, alternating
    for name, M, N, K in SHAPES[:3]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda") * 0.1
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        aux = torch.empty_like(out)
        modes = [int(m) for m in os.environ.get("PPD_MODES", "0,1").split(",")]
        t = {d: [] for d in modes}
        for rnd in range(6):
            for d in (modes if rnd % 2 == 0 else modes[::-1]):
                ext.set_gemm_deferred(d)
                for _ in range(3):
                    run(ext, x, w, b, out, aux, seed, M, N, K, 0.1)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    run(ext, x, w, b, out, aux, seed, M, N, K, 0.1)
                e.record()
                torch.cuda.synchronize()
                t[d].append(s.elapsed_time(e) / 10)
        fl = 2.0 * M * N * K
        label = {0: "one-pass", 1: "deferred", 2: "deferred, no units (timing only)"}
        print(f"{name:8s} " + "  ".join(f"{label[d]} {statistics.median(t[d]):.4f} ms ({fl / statistics.median(t[d]) / 1e9:.0f} TF)"
                                       for d in modes), flush=True)
    ext.set_gemm_deferred(0)


if __name__ == "__main__":
    main()
