#!/usr/bin/env python3
"""LayerNorm forward with the e4m3 copy (ViT-H/14 fp8 shape, T = 65792, D = 1280, bf16 output skipped as
in the steady fp8 step) at several grid caps (workgroups per CU), interleaved rounds in one process.

  python scripts/ln_ab.py [--caps 4,8,16] [--rounds 4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--caps", default="4,8,16")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--shape", default="65792,1280")
    a = ap.parse_args()
    ext = _ext.ext()
    T, D = (int(v) for v in a.shape.split(","))
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    w, b = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda") * 0.1
    q = torch.empty(T, D, dtype=torch.uint8, device="cuda")
    qs = torch.tensor([60.0], device="cuda")
    am = torch.zeros(1, dtype=torch.int32, device="cuda")
    caps = [int(c) for c in a.caps.split(",")]
    ref = None
    res = {c: [] for c in caps}
    for r in range(a.rounds):
        for c in (caps if r % 2 == 0 else caps[::-1]):
            ext.set_ln_fwd_q8_grid(c)
            for _ in range(3):
                ext.layernorm_fwd_q8(x, w, b, 1e-6, T, D, q, qs, am, True)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                ext.layernorm_fwd_q8(x, w, b, 1e-6, T, D, q, qs, am, True)
            e.record()
            torch.cuda.synchronize()
            res[c].append(s.elapsed_time(e) / 20 * 1000)
            if ref is None:
                ref = q.clone()
            elif not torch.equal(ref, q):
                raise SystemExit(f"cap {c}: output differs")
    ext.set_ln_fwd_q8_grid(4)
    gb = (T * D * 2 + T * D) / 1e9
    for c in caps:
        t = sorted(res[c])[len(res[c]) // 2]
        print(f"ln_fwd_q8 T{T} D{D} cap {c}/CU: median {t:.1f} us (best {min(res[c]):.1f}), {gb / t * 1e6 / 1e3:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
