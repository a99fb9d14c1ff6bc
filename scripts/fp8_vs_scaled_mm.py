#!/usr/bin/env python3
"""The fp8 GEMMs of a ViT-H/14 training step (batch 256, T = 65792 tokens) against
torch._scaled_mm (hipBLASLt fp8) on the same e4m3 / e5m2 operands and per-tensor scales,
interleaved in one process (alternating order per round).

  python scripts/fp8_vs_scaled_mm.py [--batch 256] [--rounds 4]

Rows: forward (e4m3 x e4m3 -> bf16 + bias [+ GELU epilogue]), dgrad (e5m2 grad x e4m3 W^T -> bf16),
weight gradient (e5m2 dy^T x e4m3 x over the tokens -> fp32, ours: split-K + ordered reduction).
torch._scaled_mm computes the plain scaled product (no bias / GELU / dropout / fp8 copy), so a ratio
> 1 on an epilogue row means our fused epilogue costs less than hipBLASLt's bare product. Also
reports the max relative difference of the products (same operands, fp32 accumulation both).
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


def timeit(fn, iters=10, warmup=3):
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


def q8(x: torch.Tensor, dtype):
    """per-tensor scaled fp8 copy (uint8 view for our kernels, typed view for torch) + dequant scale"""
    amax = x.abs().max().float().clamp(min=1e-12)
    fmax = torch.finfo(dtype).max
    s = fmax / amax
    t = (x.float() * s).clamp(-fmax, fmax).to(dtype)
    return t, (1.0 / s).reshape(1).float()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--persistent", type=int, default=None, help="ext.set_fp8_persistent mode (A/B)")
    a = ap.parse_args()
    if a.persistent is not None:
        _ext.ext().set_fp8_persistent(a.persistent)
        print(f"# fp8 persistent GEMM mode {a.persistent}", flush=True)
    dev = "cuda"
    D, M, N = 1280, 5120, 257
    T = a.batch * N
    torch.manual_seed(0)
    ext = _ext.ext()
    e4, e5 = torch.float8_e4m3fn, torch.float8_e5m2
    x = torch.randn(T, D, device=dev)
    h = torch.randn(T, M, device=dev)
    g3 = torch.randn(T, 3 * D, device=dev) * 1e-3
    gd = torch.randn(T, D, device=dev) * 1e-3
    w = {n: torch.randn(o, i, device=dev) * 0.02 for n, (o, i) in
         {"qkv": (3 * D, D), "out": (D, D), "fc1": (M, D), "fc2": (D, M)}.items()}
    x8, xs = q8(x, e4)
    h8, hs = q8(h, e4)
    g38, g3s = q8(g3, e5)
    gd8, gds = q8(gd, e5)
    w8 = {n: q8(v, e4) for n, v in w.items()}
    wt8 = {n: q8(v.t().contiguous(), e4) for n, v in w.items()}
    bias = {n: torch.randn(v.shape[0], device=dev) for n, v in w.items()}
    u8 = lambda t: t.view(torch.uint8)  # noqa: E731
    aux = torch.empty(T, M, dtype=torch.bfloat16, device=dev)
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    ws_out = {n: torch.zeros(v.shape, device=dev) for n, v in w.items()}

    def sm(a8, as_, b8t, bs, out_dtype=torch.bfloat16):
        return torch._scaled_mm(a8, b8t, scale_a=as_, scale_b=bs, out_dtype=out_dtype)

    cases = [
        # name, flops, ours, torch._scaled_mm, (our output getter, reference getter) for the accuracy check
        ("qkv fwd  +bias", 2.0 * T * 3 * D * D,
         lambda: F8.linear_fwd_fp8(u8(x8), xs, u8(w8["qkv"][0]), w8["qkv"][1], bias["qkv"]),
         lambda: sm(x8, xs, w8["qkv"][0].t(), w8["qkv"][1])),
        ("out fwd  +bias", 2.0 * T * D * D,
         lambda: F8.linear_fwd_fp8(u8(x8), xs, u8(w8["out"][0]), w8["out"][1], bias["out"]),
         lambda: sm(x8, xs, w8["out"][0].t(), w8["out"][1])),
        ("fc1 fwd  +bias+GELU+drop+aux", 2.0 * T * M * D,
         lambda: F8.linear_fwd_fp8(u8(x8), xs, u8(w8["fc1"][0]), w8["fc1"][1], bias["fc1"], gelu_aux=aux, drop=(seed, 3 << 32, 0.1)),
         lambda: sm(x8, xs, w8["fc1"][0].t(), w8["fc1"][1])),
        ("fc2 fwd  +bias", 2.0 * T * M * D,
         lambda: F8.linear_fwd_fp8(u8(h8), hs, u8(w8["fc2"][0]), w8["fc2"][1], bias["fc2"]),
         lambda: sm(h8, hs, w8["fc2"][0].t(), w8["fc2"][1])),
        ("qkv dgrad", 2.0 * T * 3 * D * D,
         lambda: F8.linear_dgrad_fp8(u8(g38), g3s, u8(wt8["qkv"][0]), wt8["qkv"][1]),
         lambda: sm(g38, g3s, wt8["qkv"][0].t(), wt8["qkv"][1])),
        ("fc1 dgrad (K = 5120)", 2.0 * T * M * D,
         lambda: F8.linear_dgrad_fp8(u8(h8), hs, u8(wt8["fc1"][0]), wt8["fc1"][1]),
         lambda: sm(h8, hs, wt8["fc1"][0].t(), wt8["fc1"][1])),
        ("out dgrad", 2.0 * T * D * D,
         lambda: F8.linear_dgrad_fp8(u8(gd8), gds, u8(wt8["out"][0]), wt8["out"][1]),
         lambda: sm(gd8, gds, wt8["out"][0].t(), wt8["out"][1])),
    ]
    # weight gradients: ours reads the row-major fp8 copies as mn-contiguous operands (split-K + ordered
    # reduction); torch._scaled_mm needs a row-major A and a column-major B: dy^T (a transposed copy) x x
    g3t8 = g38.t().contiguous()
    gdt8 = gd8.t().contiguous()
    xcm = x8.t().contiguous().t()  # column-major [T, D]
    cases += [
        ("qkv wgrad", 2.0 * T * 3 * D * D, lambda: _wgrad(ext, g38, x8, g3s, xs, ws_out["qkv"]),
         lambda: sm(g3t8, g3s, xcm, xs, torch.float32)),
        ("out wgrad", 2.0 * T * D * D, lambda: _wgrad(ext, gd8, x8, gds, xs, ws_out["out"]),
         lambda: sm(gdt8, gds, xcm, xs, torch.float32)),
    ]
    ok = []
    for c in cases:  # torch._scaled_mm may not take every operand format / output type on this build
        try:
            c[3]()
            ok.append(c)
        except Exception as e:  # noqa: BLE001
            print(f"{c[0]:30s} torch._scaled_mm unavailable: {str(e).splitlines()[0][:120]}", flush=True)
            ok.append((c[0], c[1], c[2], None))
    cases = ok
    res = {}
    for rnd in range(a.rounds):
        for name, fl, ours, lib in cases:
            order = [("ours", ours), ("lib", lib)] if rnd % 2 == 0 else [("lib", lib), ("ours", ours)]
            for vn, fn in order:
                if fn is None:
                    continue
                res.setdefault((name, vn), []).append(timeit(fn))
    print(f"# ViT-H/14 fp8 GEMMs, batch {a.batch} (T = {T}), {a.rounds} rounds; median ms, TFLOP/s", flush=True)
    for name, fl, ours, lib in cases:
        to = statistics.median(res[(name, "ours")])
        if lib is None:
            print(f"{name:30s} ours {to:7.3f} ms {fl / to / 1e9:7.1f} TF", flush=True)
            continue
        tl = statistics.median(res[(name, "lib")])
        print(f"{name:30s} ours {to:7.3f} ms {fl / to / 1e9:7.1f} TF | torch._scaled_mm {tl:7.3f} ms "
              f"{fl / tl / 1e9:7.1f} TF | x{tl / to:5.2f}", flush=True)
    # accuracy of the plain products (qkv fwd without bias: ours - bias vs scaled_mm)
    yo = F8.linear_fwd_fp8(u8(x8), xs, u8(w8["qkv"][0]), w8["qkv"][1]).float()
    yl = sm(x8, xs, w8["qkv"][0].t(), w8["qkv"][1]).float()
    print(f"qkv fwd product: max |ours - scaled_mm| / max |scaled_mm| = {(yo - yl).abs().max().item() / yl.abs().max().item():.2e}",
          flush=True)


def _wgrad(ext, dy8, x8, dys, xs, out):
    T, N = dy8.shape
    K = x8.shape[1]
    splits = G.wgrad_splits(T, N, K, 12)
    ksplit = max(128, (T // splits + 127) // 128 * 128)
    nsplit = (T + ksplit - 1) // ksplit
    ws = G._workspace(nsplit * N * K, dy8.device)[:nsplit * N * K].view(nsplit, N, K)
    ext.gemm_fp8_wgrad_mn(dy8.view(torch.uint8), x8.view(torch.uint8), ws, N, K, T, dys, xs, ksplit)
    ext.splitk_reduce(ws, nsplit, out, False)
    return out


if __name__ == "__main__":
    main()
