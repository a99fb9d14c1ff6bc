#!/usr/bin/env python3
"""Run the attention forward + backward a few times at BASELINE model shapes (for rocprofv3 --pmc /
--kernel-trace passes; scripts/pmc_attn.sh).

  python scripts/attn_probe.py --shapes h14,l16_384 --iters 3
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

SHAPES = {"l16_384": (128, 577, 16, 64), "h14": (256, 257, 16, 80), "b16": (256, 197, 12, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="h14,l16_384")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    ext = _ext.ext()
    for name in a.shapes.split(","):
        B, N, H, dh = SHAPES[name]
        qkv = torch.randn(B * N, 3 * H * dh, device="cuda", dtype=torch.bfloat16)
        for _ in range(a.iters):
            o, lse = ext.attn_fwd(qkv, B, N, H, dh ** -0.5)
        do = torch.randn_like(o)
        for _ in range(a.iters):
            ext.attn_bwd(do, qkv, o, lse, B, N, H, dh ** -0.5)
        torch.cuda.synchronize()
        print(f"{name}: B{B} N{N} H{H} dh{dh} x{a.iters}", flush=True)


if __name__ == "__main__":
    main()
