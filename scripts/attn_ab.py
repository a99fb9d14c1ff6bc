#!/usr/bin/env python3
"""Attention kernels at the BASELINE model shapes: forward (and backward) time / TFLOP/s, optionally
A/B over a kernel switch, interleaved in one process (variant order alternates per round).

  python scripts/attn_ab.py                  # ViT-L/16 384 px (N 577, dh 64), ViT-H/14 (N 257, dh 80), ViT-B/16
  python scripts/attn_ab.py --ab fwd_qg      # tiled forward: 2 query groups per wave vs 1 (round-3 form)
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # PVR_PKG_ROOT: an A/B build
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

SHAPES = {"l16_384": (128, 577, 16, 64), "h14": (256, 257, 16, 80), "b16": (256, 197, 12, 64),
          "h14_dh64": (256, 257, 20, 64), "h14_dh96": (256, 257, 13, 96), "h14_dh128": (256, 257, 10, 128)}  # D ~ 1280 at other head dims


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="l16_384,h14,b16")
    ap.add_argument("--ab", default="", help="'fwd_qg': tiled forward with 2 vs 1 query groups per wave")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--bwd", action="store_true", help="also time the backward")
    a = ap.parse_args()
    ext = _ext.ext()
    variants = [("", lambda: None)]
    if a.ab == "fwd_qg":
        variants = [("qg2", lambda: ext.set_attn_fwd_qg(2)), ("qg1", lambda: ext.set_attn_fwd_qg(1))]
    elif a.ab == "hqf":
        variants = [("hqf2", lambda: ext.set_attn_fwd_head_qf(2)), ("hqf1", lambda: ext.set_attn_fwd_head_qf(1))]
    elif a.ab == "prepxcd":  # backward pre-pass: XCD-contiguous vs round-robin (batch, head) pairs
        variants = [("prep_xcd", lambda: ext.set_attn_prep_xcd(1)), ("prep_rr", lambda: ext.set_attn_prep_xcd(0))]
    res = {}
    data = {}
    for name in a.shapes.split(","):
        B, N, H, dh = SHAPES[name]
        qkv = torch.randn(B * N, 3 * H * dh, device="cuda", dtype=torch.bfloat16)
        o, lse = ext.attn_fwd(qkv, B, N, H, dh ** -0.5)
        data[name] = (qkv, torch.randn_like(o), o, lse)
    for rnd in range(a.rounds):
        for name in a.shapes.split(","):
            B, N, H, dh = SHAPES[name]
            qkv, do, o, lse = data[name]
            order = variants if rnd % 2 == 0 else variants[::-1]
            for vn, setv in order:
                setv()
                res.setdefault((name, "fwd", vn), []).append(timeit(lambda: ext.attn_fwd(qkv, B, N, H, dh ** -0.5)))
                if a.bwd:
                    res.setdefault((name, "bwd", vn), []).append(timeit(lambda: ext.attn_bwd(do, qkv, o, lse, B, N, H, dh ** -0.5)))
    ext.set_attn_fwd_qg(0)
    ext.set_attn_fwd_head_qf(1)
    ext.set_attn_prep_xcd(0)
    for name in a.shapes.split(","):
        B, N, H, dh = SHAPES[name]
        fl = 4.0 * B * H * N * N * dh
        for vn, _ in variants:
            v = res[(name, "fwd", vn)]
            t = statistics.median(v)
            print(f"attn fwd {name:8s} B{B} N{N} H{H} dh{dh} {vn:4s} {t:7.3f} ms (min {min(v):.3f}) {fl / t / 1e9:6.1f} TF", flush=True)
        if a.bwd:
            for vn in sorted({k[2] for k in res if k[0] == name and k[1] == "bwd"}):
                t = statistics.median(res[(name, "bwd", vn)])
                print(f"attn bwd {name:8s} B{B} N{N} H{H} dh{dh} {vn:4s} {t:7.3f} ms {2.5 * fl / t / 1e9:6.1f} TF", flush=True)


if __name__ == "__main__":
    main()
