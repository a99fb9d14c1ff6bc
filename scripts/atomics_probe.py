#!/usr/bin/env python3
"""Cost of the column-reduction atomics in the fused kernels at ViT-B/16 b256 shapes: each kernel
timed with and without its f32 column-sum outputs (LayerNorm dgamma/dbeta/dsum, the dGELU GEMM's
fused bias gradient, the patch-embedding backward)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402

ext = _ext.ext()
dev = "cuda"
B, ntok, D, M = int(os.environ.get("PB", 256)), 197, 768, 3072
T = B * ntok


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)  # noqa: E731
dy, x, dres = bf(T, D), bf(T, D), bf(T, D)
mean, rstd = torch.randn(T, device=dev), torch.rand(T, device=dev) + 0.5
w = torch.rand(D, device=dev)
dx, dz = torch.empty_like(dy), torch.empty_like(dy)
dw, db, ds = torch.zeros(D, device=dev), torch.zeros(D, device=dev), torch.zeros(D, device=dev)
seed = torch.tensor([7], dtype=torch.int64, device=dev)
print(f"ln_bwd  full (dw, db, dsum, dz): {timed(lambda: ext.layernorm_bwd(dy, D, x, D, mean, rstd, w, dres, D, dx, D, dw, db, T, ds, dz, seed, 5, 0.1)):7.1f} us")
print(f"ln_bwd  no column sums (dz):    {timed(lambda: ext.layernorm_bwd(dy, D, x, D, mean, rstd, w, dres, D, dx, D, None, None, T, None, dz, seed, 5, 0.1)):7.1f} us")
print(f"ln_bwd  dw, db only:            {timed(lambda: ext.layernorm_bwd(dy, D, x, D, mean, rstd, w, dres, D, dx, D, dw, db, T)):7.1f} us")
print(f"ln_bwd  nothing extra:          {timed(lambda: ext.layernorm_bwd(dy, D, x, D, mean, rstd, w, None, D, dx, D, None, None, T)):7.1f} us")

r, w2, u = bf(T, D), (torch.randn(D, M, device=dev) * 0.02).to(torch.bfloat16), bf(T, M)
w2t = w2.t().contiguous()
cs = torch.zeros(M, device=dev)
print(f"fc2 dgrad dGELU + colsum:       {timed(lambda: G.linear_dgrad(r, w2, dgelu_aux=u, wt=w2t, colsum=cs)):7.1f} us")
print(f"fc2 dgrad dGELU:                {timed(lambda: G.linear_dgrad(r, w2, dgelu_aux=u, wt=w2t)):7.1f} us")
print(f"fc2 dgrad plain:                {timed(lambda: G.linear_dgrad(r, w2, wt=w2t)):7.1f} us")

qkv = bf(T, 3 * D)
bq = torch.zeros(3 * D, device=dev)
print(f"colsum [T, 2304]:               {timed(lambda: G.bias_grad(qkv, bq)):7.1f} us")

dE = bf(B, ntok, D)
gpos, gcls, gb = torch.zeros(ntok * D, device=dev), torch.zeros(D, device=dev), torch.zeros(D, device=dev)
dconv = torch.empty(B * (ntok - 1), D, dtype=torch.bfloat16, device=dev)
print(f"patch_bwd B{B} (drop 0.1):      {timed(lambda: ext.patch_bwd(dE, B, ntok, D, gpos, gcls, dconv, gb, seed, 3, 0.1)):7.1f} us")
