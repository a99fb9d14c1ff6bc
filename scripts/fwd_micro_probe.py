#!/usr/bin/env python3
"""Forward-only and backward-only time of the fused ViT-B/16 b256 step, single stream vs the
two-stream micro-batched blocks (PVR_MICRO A/B split by phase)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd.models import vit  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import fused_vit  # noqa: E402
from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("PB", 256))
m = vit("vit_b16", num_classes=1000).to(dev).train()
x = torch.rand(B, 3, 224, 224, device=dev)
y = torch.randint(0, 1000, (B,), device=dev)
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
for micro in (1, 2, 1, 2):
    fused_vit.MICRO = micro
    fused_vit.MICRO_MIN_IMAGES = 32
    tf = tb = 0.0
    for it in range(8):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        loss = cross_entropy(m(x), y)
        e1.record()
        loss.backward()
        e2.record()
        torch.cuda.synchronize()
        if it >= 3:
            tf += e0.elapsed_time(e1) / 5
            tb += e1.elapsed_time(e2) / 5
        for p in m.parameters():
            p.grad = None
    print(f"MICRO={micro}: forward {tf:6.2f} ms  backward {tb:6.2f} ms", flush=True)
