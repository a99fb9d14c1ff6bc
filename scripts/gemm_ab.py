#!/usr/bin/env python3
"""Every GEMM of a ViT training step exactly as the step calls it (default tile selection, fused
epilogues), timed against hipBLASLt (torch.matmul on the same bf16 operands, plain product) and
optionally A/B'd over a switch of ours, interleaved in one process (rounds x variants).

  python scripts/gemm_ab.py                     # ViT-B/16 batch 256 (T = 50432)
  python scripts/gemm_ab.py --ab tail           # split-K tail of the last dispatch round on / off
  python scripts/gemm_ab.py --ab skfix --only wgrad   # weight gradients: in-launch split-K reduction on / off
  python scripts/gemm_ab.py --model vit_h14 --batch 256

Prints one line per (GEMM, variant): median / min ms over the rounds, TFLOP/s, ratio vs hipBLASLt.
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # PVR_PKG_ROOT: an A/B build
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402

SHAPES = {"vit_b16": (768, 3072, 197), "vit_l16": (1024, 4096, 577), "vit_h14": (1280, 5120, 257)}


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


def cases(T, D, M, dev):
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    x = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
    h = torch.randn(T, M, device=dev, dtype=torch.bfloat16)
    r = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
    d3 = torch.randn(T, 3 * D, device=dev, dtype=torch.bfloat16)
    u = torch.empty(T, M, device=dev, dtype=torch.bfloat16)
    w = {n: (torch.randn(o, i, device=dev) * 0.02).to(torch.bfloat16)
         for n, (o, i) in {"qkv": (3 * D, D), "out": (D, D), "fc1": (M, D), "fc2": (D, M)}.items()}
    wt = {n: v.t().contiguous() for n, v in w.items()}
    b = {n: torch.randn(v.shape[0], device=dev) for n, v in w.items()}
    cs = torch.zeros(M, device=dev)
    ws = torch.zeros(M, D, device=dev)
    drop = lambda k: (seed, k << 32, 0.1)  # noqa: E731
    return [
        # name, flops, ours, hipBLASLt (plain product of the same operands)
        ("qkv fwd   bias", 2.0 * T * 3 * D * D, lambda: G.linear_fwd(x, w["qkv"], b["qkv"]), lambda: x @ w["qkv"].t()),
        ("out fwd   bias+resid", 2.0 * T * D * D, lambda: G.linear_fwd(x, w["out"], b["out"], resid=r), lambda: x @ w["out"].t()),
        ("fc1 fwd   bias+GELU+drop+aux", 2.0 * T * M * D,
         lambda: G.linear_fwd(x, w["fc1"], b["fc1"], gelu_aux=u, drop=drop(3)), lambda: x @ w["fc1"].t()),
        ("fc2 fwd   bias+drop+resid", 2.0 * T * M * D,
         lambda: G.linear_fwd(h, w["fc2"], b["fc2"], resid=r, drop=drop(4)), lambda: h @ w["fc2"].t()),
        ("fc2 dgrad dGELU+colsum", 2.0 * T * M * D,
         lambda: G.linear_dgrad(r, w["fc2"], dgelu_aux=u, wt=wt["fc2"], colsum=cs), lambda: r @ w["fc2"]),
        ("fc2 dgrad dGELU", 2.0 * T * M * D,
         lambda: G.linear_dgrad(r, w["fc2"], dgelu_aux=u, wt=wt["fc2"]), lambda: r @ w["fc2"]),
        ("fc1 fwd   bias+GELU+aux", 2.0 * T * M * D,
         lambda: G.linear_fwd(x, w["fc1"], b["fc1"], gelu_aux=u), lambda: x @ w["fc1"].t()),
        ("fc1 fwd   bias", 2.0 * T * M * D, lambda: G.linear_fwd(x, w["fc1"], b["fc1"]), lambda: x @ w["fc1"].t()),
        ("colsum    dU (bias grad pass)", 2.0 * T * M * D, lambda: G.bias_grad(h, cs), lambda: h.sum(0, dtype=torch.float32)),
        ("fc1 dgrad", 2.0 * T * M * D, lambda: G.linear_dgrad(h, w["fc1"], wt=wt["fc1"]), lambda: h @ w["fc1"]),
        ("out dgrad", 2.0 * T * D * D, lambda: G.linear_dgrad(r, w["out"], wt=wt["out"]), lambda: r @ w["out"]),
        ("qkv dgrad", 2.0 * T * 3 * D * D, lambda: G.linear_dgrad(d3, w["qkv"], wt=wt["qkv"]), lambda: d3 @ w["qkv"]),
        ("fc1 wgrad", 2.0 * T * M * D, lambda: G.linear_wgrad(h, x, ws), lambda: h.t() @ x),
        ("fc2 wgrad", 2.0 * T * M * D, lambda: G.linear_wgrad(r, h, ws.view(D, M)), lambda: r.t() @ h),
        ("qkv wgrad", 2.0 * T * 3 * D * D, lambda: G.linear_wgrad(d3, x, ws.view(-1)[:3 * D * D].view(3 * D, D)), lambda: d3.t() @ x),
        ("out wgrad", 2.0 * T * D * D, lambda: G.linear_wgrad(r, x, ws.view(-1)[:D * D].view(D, D)), lambda: r.t() @ x),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16", choices=sorted(SHAPES))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--ab", default="", help="'tail': split-K tail on / off")
    ap.add_argument("--only", default="", help="comma-separated substrings of case names")
    a = ap.parse_args()
    D, M, N = SHAPES[a.model]
    T = a.batch * N
    dev = "cuda"
    torch.manual_seed(0)
    ext = _ext.ext()
    variants = [("", lambda: None)]
    if a.ab == "tail":
        variants = [("tail on ", lambda: ext.set_gemm_tail(True)), ("tail off", lambda: ext.set_gemm_tail(False))]
    elif a.ab == "skfix":
        # weight gradients: in-launch split-K reduction vs the separate reduce pass
        variants = [("skfix on", lambda: setattr(G, "SPLITK_FIXUP", True)), ("skfixoff", lambda: setattr(G, "SPLITK_FIXUP", False))]
    elif a.ab.startswith("tiles:"):
        # tiles:def,7,8 - the default tile selection vs forced tile configs (every case)
        def force(t):
            return lambda: setattr(G, "FORCE_TILE", None if t == "def" else int(t))
        variants = [(f"t{t:6s}", force(t)) for t in a.ab.split(":", 1)[1].split(",")]
    cs = [c for c in cases(T, D, M, dev) if not a.only or any(s in c[0] for s in a.only.split(","))]
    res = {}
    for rnd in range(a.rounds):
        for name, fl, ours, lib in cs:
            # variant order alternates per round (A B lib, then lib B A, ...): a fixed order biased the
            # comparison by ~10 % on GEMMs the switch does not even touch (clock / power history)
            order = variants if rnd % 2 == 0 else variants[::-1]
            if rnd % 2:
                res.setdefault((name, "lib"), []).append(timeit(lib))
            for vn, setv in order:
                setv()
                res.setdefault((name, vn), []).append(timeit(ours))
            if rnd % 2 == 0:
                res.setdefault((name, "lib"), []).append(timeit(lib))
    ext.set_gemm_tail(True)
    G.FORCE_TILE = None
    print(f"# {a.model} batch {a.batch} (T = {T}), {a.rounds} rounds; median (min) ms, TFLOP/s at the median", flush=True)
    for name, fl, _, _ in cs:
        tl = statistics.median(res[(name, "lib")])
        print(f"{name:30s} hipBLASLt {tl:7.3f} ms {fl / tl / 1e9:7.1f} TF", flush=True)
        for vn, _ in variants:
            v = res[(name, vn)]
            t = statistics.median(v)
            print(f"{name:30s} ours {vn:8s} {t:7.3f} ({min(v):7.3f}) ms {fl / t / 1e9:7.1f} TF  x{tl / t:5.2f} vs hipBLASLt",
                  flush=True)


if __name__ == "__main__":
    main()
