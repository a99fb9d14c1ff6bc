#!/usr/bin/env python3
"""Phase-segment cycles of the ping-pong GEMM K loop (diagnostic build -DPVR_GEMM_PHASE_STAMPS, selected
with PVR_PKG_ROOT): per wave, s_memtime sums over every phase of the K loop, printed as the median
over waves per phase (4 phases per 64-deep K-tile). Shapes: the ViT-B/16 b256 qkv weight gradient
(mn-contiguous operands, split-K partials: tile 14) and the qkv forward on the one-tile-per-workgroup
form (k-contiguous: tile 12), same FLOPs.

  PVR_PKG_ROOT=ab_gst python scripts/gemm_phase_stamps.py
  ONLY_TYPE=0 PVR_PKG_ROOT=ab_t0 python scripts/gemm_phase_stamps.py   # -DPVR_GEMM_PHASE_ONLY_TYPE=0 build
"""
from __future__ import annotations

import math
import os
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402

SEG = ["reads issue", "DMA issue", "vmcnt wait", "barrier 1", "lgkmcnt wait", "MFMA issue", "barrier 2", "K loop total"]
if os.environ.get("PPT"):  # build with -DPVR_GEMM_PHASE_BY_TYPE too: per phase type (4 per K-tile)
    SEG = ["phase (0,0) whole", "phase (0,1) whole", "phase (1,1) whole", "phase (1,0) whole",
           "phase (0,0) R-part", "phase (0,1) R-part", "phase (1,1) R-part", "phase (1,0) R-part"]


def report(name, dbg, nphases):
    d = dbg.view(-1, 8).double()
    if not os.environ.get("PPT"):
        d = d[d[:, 7] > 0]
    if os.environ.get("PPT"):
        d = d[d[:, 0] > 0]
        med = d.median(0).values / (nphases / 4)
        print(f"# {name}: {d.shape[0]} waves, cycles per phase of each type (median over waves)", flush=True)
        for k, s in enumerate(SEG):
            print(f"  {s:20s} {med[k].item():8.1f}", flush=True)
        return
    med = d.median(0).values / nphases
    if os.environ.get("ONLY_TYPE"):  # build with -DPVR_GEMM_PHASE_ONLY_TYPE=t: a quarter of the phases summed
        med[:7] *= 4
        name += f" [phase type {os.environ['ONLY_TYPE']} only]"
    print(f"# {name}: {d.shape[0]} waves, cycles per phase (median over waves; 16 MFMAs per wave per phase)", flush=True)
    for k, s in enumerate(SEG):
        print(f"  {s:14s} {med[k].item():8.1f}", flush=True)
    print(f"  {'sum 0-6':14s} {med[:7].sum().item():8.1f}", flush=True)


def main():
    ext = _ext.ext()
    T, D = 50432, 768
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    d3 = torch.randn(T, 3 * D, device="cuda").to(torch.bfloat16)
    N, K = 3 * D, D
    splits = G.wgrad_splits(T, N, K, 12)
    ksplit = math.ceil(math.ceil(T / splits) / 64) * 64
    nsplit = math.ceil(T / ksplit)
    ws = torch.empty(nsplit, N, K, device="cuda")
    ntiles = math.ceil(N / 256) * math.ceil(K / 256)
    dbg = torch.zeros(ntiles * nsplit * 64, dtype=torch.int64, device="cuda")
    for _ in range(4):
        ext.gemm(d3, False, x, False, ws, N, K, T, 4, None, None, None, 0, None, 0, 0, 0, None, 0, 0.0, ksplit, 14, dbg=dbg)
    torch.cuda.synchronize()
    report(f"qkv wgrad M{N} N{K} K{T} ({nsplit} splits of {ksplit})", dbg, 4 * (ksplit // 64))
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(N, device="cuda")
    out = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    ntiles = math.ceil(T / 256) * math.ceil(N / 256)
    dbg = torch.zeros(ntiles * 64, dtype=torch.int64, device="cuda")
    for _ in range(4):
        ext.gemm(x, True, w, True, out, T, N, K, 0, b, None, None, 0, None, 0, 0, 0, None, 0, 0.0, 0, 12, dbg=dbg, tail_limit=-1)
    torch.cuda.synchronize()
    report(f"qkv fwd M{T} N{N} K{K} (tile 12, bias epilogue)", dbg, 4 * (K // 64))


if __name__ == "__main__":
    main()
