#!/usr/bin/env python3
"""Per-tensor gradient error of the fp8 backward against the bf16 backward of the same fp8-forward model,
e4m3 vs e5m2 gradients, at a full BASELINE model size (default ViT-H/14, 224 px, random init, a
synthetic batch). Same method as tests/kernel_checks.py::check_vit_fp8_grad_formats: for each format the
scaling state starts fresh, the first backward calibrates every slot, the second is measured.

  python scripts/fp8_grad_error.py [--model vit_h14] [--batch 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd.models import vit  # noqa: E402
from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_h14")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--classes", type=int, default=1000)
    a = ap.parse_args()
    torch.manual_seed(0)
    m = vit(a.model, num_classes=a.classes, mlp_dropout=0.0, embedding_dropout=0.0).cuda()
    x = torch.rand(a.batch, 3, 224, 224, device="cuda")
    y = torch.randint(0, a.classes, (a.batch,), device="cuda")
    names = [n for n, p in m.named_parameters() if "encoder" in n]

    def grads(dgrad, fmt):
        m.enable_fp8(dgrad=dgrad, wgrad=dgrad, grad_fmt=fmt)
        for _ in range(2):
            m.zero_grad(set_to_none=False)
            cross_entropy(m(x), y).backward()
        torch.cuda.synchronize()
        return {n: p.grad.float().clone() for n, p in m.named_parameters() if n in names}

    ref = grads(False, "e5m2")
    res = {}
    for fmt in ("e5m2", "e4m3"):
        g = grads(True, fmt)
        e = {n: ((g[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-30)).item() for n in names}
        res[fmt] = e
        del g
    kinds = {}
    for n in names:
        k = ".".join(n.split(".")[-3:]) if "mlp" in n or "attention" in n else n.split(".")[-2] + "." + n.split(".")[-1]
        kinds.setdefault(k, []).append(n)
    print(f"{a.model} batch {a.batch}: mean per-tensor rel-L2 of the encoder gradients vs the bf16 backward")
    print("| parameter kind | tensors | e5m2 | e4m3 | ratio |")
    print("|---|---:|---:|---:|---:|")
    for k, ns in sorted(kinds.items()):
        e5 = sum(res["e5m2"][n] for n in ns) / len(ns)
        e4 = sum(res["e4m3"][n] for n in ns) / len(ns)
        print(f"| {k} | {len(ns)} | {e5:.4f} | {e4:.4f} | {e4 / e5:.2f} |")
    e5 = sum(res["e5m2"].values()) / len(names)
    e4 = sum(res["e4m3"].values()) / len(names)
    print(f"| all | {len(names)} | {e5:.4f} | {e4:.4f} | {e4 / e5:.2f} |")


if __name__ == "__main__":
    main()
