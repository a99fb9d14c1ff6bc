#!/usr/bin/env python3
"""Phase cycles of the attention backward's query-block loop (diagnostic build with -DPVR_ATTN_STAMPS:
``python -m pytorch_vit_paper_replication_amd.build --hipcc-flag=-DPVR_ATTN_STAMPS`` into a copy of
the package, selected with PVR_PKG_ROOT). Per wave, s_memtime cycles summed over the loop by phase;
printed as the median over waves of cycles per query block.

  PVR_PKG_ROOT=ab_stamps python scripts/attn_stamps.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402

SHAPES = {"l16_384": (128, 577, 16, 64), "h14": (256, 257, 16, 80), "n256": (256, 256, 16, 64), "b16": (256, 197, 12, 64)}
PHASES = ["wait vmcnt", "barrier", "stage issue", "S/dP", "P/dS valu", "dS write + dV/dK", "dQ", "total"]
# the persistent whole-head kernel (192 < N <= 224): one workgroup per CU walks its (batch, head) pairs
PIPE8 = ["wait + barrier", "DMA group issue", "pair switch", "S/dP", "dQ (prev block)", "next table", "P/dS + dV/dK", "loop total"]


def main():
    ext = _ext.ext()
    for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else list(SHAPES)):
        B, N, H, dh = SHAPES[name]
        qkv = torch.randn(B * N, 3 * H * dh, device="cuda", dtype=torch.bfloat16)
        o, lse = ext.attn_fwd(qkv, B, N, H, dh ** -0.5)
        do = torch.randn_like(o)
        nkb = ext.attn_bwd_key_blocks(N) if hasattr(ext, "attn_bwd_key_blocks") else (N + 255) // 256
        dbg = torch.zeros(nkb * B * H * 8 * 8, dtype=torch.int64, device="cuda")
        ext.set_attn_dbg(dbg)
        for _ in range(5):
            ext.attn_bwd(do, qkv, o, lse, B, N, H, dh ** -0.5)
        torch.cuda.synchronize()
        ext.set_attn_dbg(torch.empty(0, device="cuda"))
        d = dbg.view(-1, 8).double()
        d = d[d[:, 7] > 0]
        nqb = (N + 31) // 32
        names = PHASES
        if 192 < N <= 224 and dh == 64:  # pipe8: blocks per workgroup = pairs per CU x query blocks
            cus = torch.cuda.get_device_properties(0).multi_processor_count
            nqb *= -(-B * H // min(B * H, cus))
            names = PIPE8
        med = d.median(0).values / nqb
        print(f"# {name}: B{B} N{N} H{H} dh{dh}, {d.shape[0]} waves, cycles per query block (median over waves)", flush=True)
        for k, ph in enumerate(names):
            print(f"  {ph:18s} {med[k].item():8.0f}", flush=True)
        print(f"  {'sum of phases':18s} {med[:7].sum().item():8.0f}", flush=True)
        if names is PIPE8 and d.shape[0] % 8 == 0:  # per wave (wave 7 holds no key below N, wave 6 one fragment)
            w = d.view(-1, 8, 8).mean(0) / nqb
            for i in range(8):
                print(f"  wave {i}: " + " ".join(f"{w[i, k].item():6.0f}" for k in range(8)), flush=True)


if __name__ == "__main__":
    main()
