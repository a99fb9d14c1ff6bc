#!/usr/bin/env python3
"""Last-round tile quantisation of the N = 768 GEMMs at ViT-B/16 b256 (T = 50432 tokens).

256x256 tiles give 197 x 3 = 591 workgroups = 2.31 rounds of 256 CUs: the third round runs 79
workgroups on 256 CUs. This probe times, per GEMM shape, the whole GEMM on the ping-pong tile (12)
against a row split: the first R0 rows (a whole number of 256-row tiles filling 2 rounds) on tile
12 and the remaining rows on a smaller tile (0 = 128x128, 9 / 10 = 4-wave two-per-CU tiles).
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=30, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def fwd(x, w, b, resid, out, tile):
    T, K = x.shape
    N = w.shape[0]
    _ext.ext().gemm(x, True, w, True, out, T, N, K, G.EPI_BF16, b, resid, None, 0, None, 0, 0, 0,
                    None, 0, 0.0, 0, tile)


def dgrad(dy, wt, out, tile):
    T, N = dy.shape
    K = wt.shape[0]
    _ext.ext().gemm(dy, True, wt, True, out, T, K, N, G.EPI_BF16, None, None, None, 0, None, 0, 0, 0,
                    None, 0, 0.0, 0, tile)


def main():
    dev = "cuda"
    T = int(os.environ.get("PVR_PROBE_T", 50432))
    D, M = 768, 3072
    torch.manual_seed(0)
    tails = [int(t) for t in os.environ.get("PVR_PROBE_TAILS", "0,9,10,1,2").split(",")]
    for name, k in (("out", D), ("fc2", M), ("qkv_dgrad", 2304), ("fc1_dgrad", M)):
        x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(D, k, device=dev) * 0.02).to(torch.bfloat16)
        b = torch.randn(D, device=dev)
        r = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
        out = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * D * k
        if name.endswith("dgrad"):
            run = lambda xs, os_, tile: dgrad(xs, w, os_, tile)  # noqa: E731  (w plays W^T [K_out, N_in])
            rs = None
        else:
            run = lambda xs, os_, tile: fwd(xs, w, b, rs_cur[0], os_, tile)  # noqa: E731
            rs = r
        rs_cur = [rs]
        t12 = timeit(lambda: run(x, out, 12))
        ref = out.clone()
        print(f"{name:10s} K{k:5d} whole tile12 {t12:7.1f} us {fl / t12 / 1e6:7.1f} TF", flush=True)
        ntn = (D + 255) // 256
        for rounds in (2,):
            mt = (rounds * 256) // ntn          # 256-row tiles in the first part
            r0 = mt * 256
            if r0 >= T:
                continue
            for tail in tails:
                def split():
                    rs_cur[0] = rs[:r0] if rs is not None else None
                    run(x[:r0], out[:r0], 12)
                    rs_cur[0] = rs[r0:] if rs is not None else None
                    run(x[r0:], out[r0:], tail)
                    rs_cur[0] = rs
                ts = timeit(split)
                err = (out.float() - ref.float()).abs().max().item()
                print(f"{name:10s} split rows {r0}+{T - r0} tail tile{tail:2d} {ts:7.1f} us {fl / ts / 1e6:7.1f} TF "
                      f"x{t12 / ts:5.3f} maxdiff {err:.3g}", flush=True)
                # the tail part alone
                rs_cur[0] = rs[r0:] if rs is not None else None
                tt = timeit(lambda: run(x[r0:], out[r0:], tail))
                rs_cur[0] = rs
                print(f"{name:10s}   tail alone tile{tail:2d} {tt:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
