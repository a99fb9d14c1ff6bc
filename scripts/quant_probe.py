"""fp8 quantization pass bandwidth at ViT-H/14 b128 activation / gradient shapes (PVR_FP8_QBLOCKS A/B)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from bench_kernels import timeit  # noqa: E402

ext = _ext.ext()
T = 128 * 257
for cols, fmt in ((1280, 0), (5120, 0), (5120, 1), (3840, 1)):
    x = torch.randn(T, cols, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(T, cols, device="cuda", dtype=torch.uint8)
    qs = torch.ones(1, device="cuda")
    am = torch.zeros(1, dtype=torch.int32, device="cuda")
    t = timeit(lambda: ext.fp8_quant(x, y, qs, am, fmt))
    gb = T * cols * 3 / 1e9
    print(f"quant fmt{fmt} [{T},{cols}] blocks={os.environ.get('PVR_FP8_QBLOCKS', '256')}: {t * 1e3:.1f} us {gb / t * 1e3:.0f} GB/s", flush=True)
