#!/usr/bin/env python3
"""How much would per-32-token MX block scales improve the fp8 weight gradients? (verdict round 5, item 5)

Captures the (dy, x) operand pairs of every weight-gradient GEMM of one fused ViT backward (bf16
path, random images, a few warm-up steps of training first so the gradients are not at init), then
quantizes them the two ways the fp8 GEMM could consume them and compares each product against the
bf16 operands' exact fp32 product:
  * per-tensor: one scale per operand, amax / fp8 max (the scaling the framework's fp8 wgrad uses,
    without the delayed history: the most favourable per-tensor case);
  * MX: an E8M0 (power-of-two) scale per 32 consecutive tokens of each feature column, the OCP MX
    block the gfx950 v_mfma_scale_f32_16x16x128_f8f6f4 instruction takes per lane.
dy is e5m2, x is e4m3 (the framework's formats); and, the MXFP8 recipe's choice, dy in e4m3 too
(per-tensor and MX: the block scales give e4m3 the range e5m2 otherwise buys with a mantissa bit).
Reports rel-L2 of dW per GEMM kind.

  python scripts/mx_wgrad_study.py [--model vit_b16] [--batch 32] [--warmup-steps 20]
"""
import argparse
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

E4M3, E5M2 = torch.float8_e4m3fn, torch.float8_e5m2
FMAX = {E4M3: 448.0, E5M2: 57344.0}


def q_tensor(t: torch.Tensor, dt) -> torch.Tensor:
    """per-tensor scale: amax -> the format's max; dequantized fp32"""
    s = FMAX[dt] / t.abs().amax().clamp_min(1e-30)
    return (t * s).to(dt).float() / s


def q_mx(t: torch.Tensor, dt, block: int = 32) -> torch.Tensor:
    """[T, C] with an E8M0 scale per (32 tokens, column): 2^(ceil(log2(amax / fmax))); dequantized fp32"""
    T, C = t.shape
    Tp = (T + block - 1) // block * block
    x = torch.zeros(Tp, C, device=t.device, dtype=torch.float32)
    x[:T] = t
    xb = x.view(Tp // block, block, C)
    amax = xb.abs().amax(dim=1, keepdim=True).clamp_min(1e-30)
    e = torch.ceil(torch.log2(amax / FMAX[dt]))
    s = torch.exp2(e)
    return ((xb / s).to(dt).float() * s).view(Tp, C)[:T]


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--warmup-steps", type=int, default=20)
    a = ap.parse_args()
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import vit
    from pytorch_vit_paper_replication_amd.ops import gemm
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay

    _ext.ext()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = vit(a.model, num_classes=10).to(dev)
    opt = FusedAdam(param_groups_weight_decay(model, 0.03), lr=1e-4)
    gen = torch.Generator(device=dev).manual_seed(0)
    templates = torch.rand(10, 3, 224, 224, generator=gen, device=dev)
    for _ in range(a.warmup_steps):  # leave the init so the gradients have a training-time shape
        y = torch.randint(0, 10, (a.batch,), generator=gen, device=dev)
        x = 0.7 * templates[y] + 0.3 * torch.rand(a.batch, 3, 224, 224, generator=gen, device=dev)
        loss = cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step(clip_norm=1.0)
    captured = []
    orig = gemm.linear_wgrad

    def capture(dy, xx, out):
        captured.append((dy.detach().clone(), xx.detach().clone()))
        return orig(dy, xx, out)

    gemm.linear_wgrad = capture
    try:
        y = torch.randint(0, 10, (a.batch,), generator=gen, device=dev)
        x = 0.7 * templates[y] + 0.3 * torch.rand(a.batch, 3, 224, 224, generator=gen, device=dev)
        opt.zero_grad()
        cross_entropy(model(x), y).backward()
        torch.cuda.synchronize()
    finally:
        gemm.linear_wgrad = orig
    per_kind = defaultdict(lambda: {"tensor": [], "mx": [], "tensor43": [], "mx43": []})
    for dy, xx in captured:
        T = min(dy.shape[0], xx.shape[0])
        dy, xx = dy[:T].float(), xx[:T].float()
        kind = f"{dy.shape[1]}x{xx.shape[1]}"
        ref = dy.t() @ xx
        per_kind[kind]["tensor"].append(rel(q_tensor(dy, E5M2).t() @ q_tensor(xx, E4M3), ref))
        per_kind[kind]["mx"].append(rel(q_mx(dy, E5M2).t() @ q_mx(xx, E4M3), ref))
        per_kind[kind]["tensor43"].append(rel(q_tensor(dy, E4M3).t() @ q_tensor(xx, E4M3), ref))
        per_kind[kind]["mx43"].append(rel(q_mx(dy, E4M3).t() @ q_mx(xx, E4M3), ref))
    rows = []
    print(f"# {a.model} batch {a.batch}, {len(captured)} weight-gradient GEMMs after {a.warmup_steps} training steps; "
          "rel-L2 of dW vs the fp32 product of the bf16 operands (mean / max over the layers)")
    print("| GEMM (N x K) | count | dy e5m2, per-tensor | dy e5m2, MX | dy e4m3, per-tensor | dy e4m3, MX |")
    print("|---|---:|---:|---:|---:|---:|")
    for kind, d in sorted(per_kind.items()):
        r = {"gemm": kind, "n": len(d["tensor"])}
        cells = []
        for key in ("tensor", "mx", "tensor43", "mx43"):
            v = d[key]
            r[key + "_mean"], r[key + "_max"] = sum(v) / len(v), max(v)
            cells.append(f"{sum(v) / len(v):.4f} / {max(v):.4f}")
        rows.append(r)
        print(f"| {kind} | {r['n']} | " + " | ".join(cells) + " |")
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
