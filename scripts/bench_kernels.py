#!/usr/bin/env python3
"""Microbenchmarks of the hand-written gfx950 kernels at ViT-B/16 training shapes (batch 256 ->
T = 50432 tokens), against the vendor-library / PyTorch equivalents on the same random data:
  * GEMM fwd / dgrad / wgrad (ours, per tile config) vs torch.matmul (hipBLASLt)
  * attention fwd / bwd vs torch scaled_dot_product_attention
  * LayerNorm fwd / bwd vs torch
Prints one line per case: time (ms), TFLOP/s (or GB/s), ratio vs the library.
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tiles", default="0,12")
    ap.add_argument("--only", default="gemm,attn,ln")
    ap.add_argument("--attn-shape", default="197,12,64", help="N,H,dh of the attention cases (batch: --batch)")
    ap.add_argument("--epi-tiles", default="12,13", help="tile configs of the per-epilogue cases (--only epi)")
    ap.add_argument("--gelu-tiles", default="6,12,13", help="tile configs of the fc1 GELU case (--only epi)")
    ap.add_argument("--rounds", type=int, default=1, help="repeat the epilogue cases (interleaved A/B)")
    a = ap.parse_args()
    dev = "cuda"
    T = a.batch * 197
    D, M3, M = 768, 2304, 3072
    tiles = [int(t) for t in a.tiles.split(",")]
    torch.manual_seed(0)
    if "gemm" in a.only:
        for (n, k, name) in [(M3, D, "qkv"), (D, D, "out"), (M, D, "fc1"), (D, M, "fc2")]:
            x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
            b = torch.randn(n, device=dev)
            dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * T * n * k
            t_lib = timeit(lambda: torch.matmul(x, w.t()))
            print(f"fwd   {name:4s} T{T} N{n} K{k}  hipblaslt {t_lib:7.3f} ms {fl / t_lib / 1e9:7.1f} TF", flush=True)
            for t in tiles:
                G.FORCE_TILE = t
                tt = timeit(lambda: G.linear_fwd(x, w, b))
                print(f"fwd   {name:4s} tile{t}      ours {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF  x{t_lib / tt:5.2f}", flush=True)
            t_lib = timeit(lambda: torch.matmul(dy, w))
            print(f"dgrad {name:4s} T{T} N{k} K{n}  hipblaslt {t_lib:7.3f} ms {fl / t_lib / 1e9:7.1f} TF", flush=True)
            wt = w.t().contiguous()
            for t in tiles:
                G.FORCE_TILE = t
                tt = timeit(lambda: G.linear_dgrad(dy, w, wt=wt))
                print(f"dgrad {name:4s} tile{t}   ours(wT) {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF  x{t_lib / tt:5.2f}", flush=True)
                tt = timeit(lambda: G.linear_dgrad(dy, w, tile=t))
                print(f"dgrad {name:4s} tile{t}   ours(W)  {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF  x{t_lib / tt:5.2f}", flush=True)
            out = torch.zeros(n, k, device=dev)
            t_lib = timeit(lambda: torch.matmul(dy.t(), x))
            print(f"wgrad {name:4s} N{n} K{k} T{T}  hipblaslt {t_lib:7.3f} ms {fl / t_lib / 1e9:7.1f} TF", flush=True)
            for t in [t for t in tiles if t in (0, 6, 12)]:
                G.FORCE_TILE = t
                tt = timeit(lambda: G.linear_wgrad(dy, x, out))
                print(f"wgrad {name:4s} tile{t}      ours {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF  x{t_lib / tt:5.2f}", flush=True)
            G.FORCE_TILE = None
    if "epi" in a.only:
        # the fused epilogues exactly as the training step runs them (ViT-B/16 b256 shapes)
        seed = torch.tensor([1234], dtype=torch.int64, device=dev)
        x = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
        h = torch.randn(T, M, device=dev, dtype=torch.bfloat16)
        r = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
        w1 = (torch.randn(M, D, device=dev) * 0.02).to(torch.bfloat16)
        w2 = (torch.randn(D, M, device=dev) * 0.02).to(torch.bfloat16)
        wo = (torch.randn(D, D, device=dev) * 0.02).to(torch.bfloat16)
        b1, b2 = torch.randn(M, device=dev), torch.randn(D, device=dev)
        u = torch.empty(T, M, device=dev, dtype=torch.bfloat16)
        cs = torch.zeros(M, device=dev)
        w2t = w2.t().contiguous()
        cases = [
            ("fc1 fwd  bias+GELU+dropout+aux", 2.0 * T * M * D, lambda: G.linear_fwd(x, w1, b1, gelu_aux=u, drop=(seed, 3 << 32, 0.1))),
            ("fc1 fwd  bias only           ", 2.0 * T * M * D, lambda: G.linear_fwd(x, w1, b1)),
            ("fc2 fwd  bias+dropout+resid  ", 2.0 * T * M * D, lambda: G.linear_fwd(h, w2, b2, resid=r, drop=(seed, 4 << 32, 0.1))),
            ("out fwd  bias+resid          ", 2.0 * T * D * D, lambda: G.linear_fwd(x, wo, b2, resid=r)),
            ("fc2 dgrad dGELU+colsum (wT)  ", 2.0 * T * M * D, lambda: G.linear_dgrad(r, w2, dgelu_aux=u, wt=w2t, colsum=cs)),
        ]
        for name, fl, fn in cases:
            tt = timeit(fn)
            print(f"epi   {name} {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF", flush=True)
        wqkv = (torch.randn(M3, D, device=dev) * 0.02).to(torch.bfloat16)
        bqkv = torch.randn(M3, device=dev)
        w1t = w1.t().contiguous()
        wot = wo.t().contiguous()
        dq3, wqkvt = torch.randn(T, M3, device=dev, dtype=torch.bfloat16), wqkv.t().contiguous()
        for _round in range(a.rounds):
          for t in [int(v) for v in a.epi_tiles.split(",")]:  # one tile per workgroup / persistent / stream-K
            G.FORCE_TILE = t
            for name, fl, fn in [
                ("qkv fwd  bias            ", 2.0 * T * M3 * D, lambda: G.linear_fwd(x, wqkv, bqkv)),
                ("out fwd  bias+resid      ", 2.0 * T * D * D, lambda: G.linear_fwd(x, wo, b2, resid=r)),
                ("fc1 fwd  GELU+drop+aux   ", 2.0 * T * M * D, lambda: G.linear_fwd(x, w1, b1, gelu_aux=u, drop=(seed, 3 << 32, 0.1))),
                ("fc2 fwd  bias+drop+resid ", 2.0 * T * M * D, lambda: G.linear_fwd(h, w2, b2, resid=r, drop=(seed, 4 << 32, 0.1))),
                ("out dgrad plain (wT)     ", 2.0 * T * D * D, lambda: G.linear_dgrad(r, wo, wt=wot)),
                ("qkv dgrad plain (wT)     ", 2.0 * T * M3 * D, lambda: G.linear_dgrad(dq3, wqkv, wt=wqkvt)),
                ("fc1 dgrad plain (wT)     ", 2.0 * T * M * D, lambda: G.linear_dgrad(u, w1, wt=w1t)),
                ("fc2 dgrad dGELU+colsum   ", 2.0 * T * M * D, lambda: G.linear_dgrad(r, w2, dgelu_aux=u, wt=w2t, colsum=cs)),
            ]:
                tt = timeit(fn)
                print(f"epi   {name} tile{t} {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF", flush=True)
            G.FORCE_TILE = None
        for t in [int(v) for v in a.gelu_tiles.split(",") if v]:  # other structures for the GELU epilogue
            G.FORCE_TILE = t
            tt = timeit(lambda: G.linear_fwd(x, w1, b1, gelu_aux=u, drop=(seed, 3 << 32, 0.1)))
            G.FORCE_TILE = None
            print(f"epi   fc1 fwd GELU tile{t:<3d}            {tt:7.3f} ms {2.0 * T * M * D / tt / 1e9:7.1f} TF", flush=True)
    if "fp8" in a.only:
        from pytorch_vit_paper_replication_amd.ops import fp8 as F8

        for (T8, n, k, name) in [(T, 2304, 768, "B qkv"), (T, 3072, 768, "B fc1"), (T, 768, 3072, "B fc2"),
                                 (128 * 257, 3840, 1280, "H qkv"), (128 * 257, 5120, 1280, "H fc1"),
                                 (128 * 257, 1280, 5120, "H fc2")]:
            x = torch.randn(T8, k, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
            b = torch.randn(n, device=dev)
            fl = 2.0 * T8 * n * k
            meta = F8.Fp8Meta(2, dev, history=1)
            xq, xs = meta.quantize(x, 0, current=True)
            wq, ws = meta.quantize(w, 1, current=True)
            G.FORCE_TILE = 12
            t16 = timeit(lambda: G.linear_fwd(x, w, b))
            G.FORCE_TILE = None
            t8 = timeit(lambda: F8.linear_fwd_fp8(xq, xs, wq, ws, b))
            tq = timeit(lambda: meta.quantize(x, 0))
            t_lib = timeit(lambda: torch.matmul(x, w.t()))
            print(f"fp8 fwd {name:6s} T{T8} N{n} K{k}: bf16 {t16:.3f} ms {fl / t16 / 1e9:6.1f} TF | fp8 {t8:.3f} ms "
                  f"{fl / t8 / 1e9:6.1f} TF (x{t16 / t8:.2f}) | act quant {tq:.3f} ms | hipblaslt bf16 {t_lib:.3f} ms",
                  flush=True)
    if "attn" in a.only:
        ext = _ext.ext()
        N, H, dh = (int(v) for v in a.attn_shape.split(","))
        B, Da, sc = a.batch, H * dh, dh ** -0.5
        qkv = torch.randn(B * N, 3 * Da, device=dev, dtype=torch.bfloat16)
        fl = 4.0 * B * H * N * N * dh
        tt = timeit(lambda: ext.attn_fwd(qkv, B, N, H, sc))
        q, k, v = qkv.view(B, N, 3, H, dh).permute(2, 0, 3, 1, 4).contiguous()
        t_lib = timeit(lambda: F.scaled_dot_product_attention(q, k, v))
        print(f"attn_fwd B{B} N{N} H{H}: ours {tt:.3f} ms {fl / tt / 1e9:.1f} TF | sdpa {t_lib:.3f} ms x{t_lib / tt:.2f}", flush=True)
        o, lse = ext.attn_fwd(qkv, B, N, H, sc)
        do = torch.randn_like(o)
        tt = timeit(lambda: ext.attn_bwd(do, qkv, o, lse, B, N, H, sc))
        qr, kr, vr = (t.detach().requires_grad_(True) for t in (q, k, v))
        orf = F.scaled_dot_product_attention(qr, kr, vr)
        dor = torch.randn_like(orf)
        t_lib = timeit(lambda: torch.autograd.grad(orf, (qr, kr, vr), dor, retain_graph=True))
        print(f"attn_bwd B{B} N{N} H{H}: ours {tt:.3f} ms {2.5 * fl / tt / 1e9:.1f} TF | sdpa {t_lib:.3f} ms x{t_lib / tt:.2f}", flush=True)
        prow = ext.attn_bwd_bias_rows(B, N, H, Da)
        if prow > 0:
            part = torch.empty(B * H, prow, 192, device=dev, dtype=torch.float32)
            tb = timeit(lambda: ext.attn_bwd(do, qkv, o, lse, B, N, H, sc, None, part))
            print(f"attn_bwd+dbias B{B} N{N} H{H}: ours {tb:.3f} ms (bias partials in-kernel)", flush=True)
    if "ln" in a.only:
        ext = _ext.ext()
        x = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
        w, b = torch.ones(D, device=dev), torch.zeros(D, device=dev)
        tt = timeit(lambda: ext.layernorm_fwd(x, w, b, 1e-5, T, D))
        t_lib = timeit(lambda: F.layer_norm(x, (D,), w.bfloat16(), b.bfloat16()))
        gb = 2 * T * D * 2 / 1e9
        print(f"ln_fwd T{T} D{D}: ours {tt:.3f} ms {gb / tt * 1e3:.0f} GB/s | torch {t_lib:.3f} ms x{t_lib / tt:.2f}", flush=True)
        y, mu, rs = ext.layernorm_fwd(x, w, b, 1e-5, T, D)
        dx = torch.empty_like(x)
        dw, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        dy, dres = torch.randn_like(x), torch.randn_like(x)
        tt = timeit(lambda: ext.layernorm_bwd(dy, D, x, D, mu, rs, w, dres, D, dx, D, dw, db, T))
        print(f"ln_bwd T{T} D{D}: ours {tt:.3f} ms {4 * T * D * 2 / 1e9 / tt * 1e3:.0f} GB/s (dy, x, dres, dx distinct)", flush=True)
        dz, ds = torch.empty_like(x), torch.zeros(D, device=dev)
        seed = torch.tensor([99], dtype=torch.int64, device=dev)
        tt = timeit(lambda: ext.layernorm_bwd(dy, D, x, D, mu, rs, w, dres, D, dx, D, dw, db, T, dsum=ds, dz=dz, seed=seed,
                                              seed_offset=2 << 32, drop_p=0.1))
        print(f"ln_bwd+dz T{T} D{D}: ours {tt:.3f} ms {5 * T * D * 2 / 1e9 / tt * 1e3:.0f} GB/s (linked dropout backward)", flush=True)
        tt = timeit(lambda: dx.copy_(dy))
        print(f"copy bf16 T{T} D{D}: {tt:.3f} ms {2 * T * D * 2 / 1e9 / tt * 1e3:.0f} GB/s (torch copy_, reference)", flush=True)


if __name__ == "__main__":
    main()
