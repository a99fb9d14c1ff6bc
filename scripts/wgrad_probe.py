"""Split-K weight-gradient GEMM epilogue variants at the ViT-B/16 b256 shapes (T = 50,432):
  t12 atomic : ping-pong, unstaged f32 atomics (4 rows x 64 B per wave instruction)
  t14 atomic : ping-pong, LDS-staged dense f32 atomics (one 256-B row run per wave instruction)
  t14 store  : ping-pong, LDS-staged f32 partial stores to a [splits, N, K] workspace + reduce kernel
Each variant is checked against a fp32 torch reference first."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

ext = _ext.ext()
T = int(os.environ.get("PROBE_T", 50432))
torch.manual_seed(0)
for (N, K, name) in [(2304, 768, "qkv"), (768, 768, "out"), (3072, 768, "fc1"), (768, 3072, "fc2")]:
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = torch.zeros(N, K, device="cuda")
    for mul in (1, 2):
        s = G.wgrad_splits(T, N, K, 12) * mul
        ks = math.ceil(math.ceil(T / s) / 64) * 64
        ns = math.ceil(T / ks)
        ws = torch.empty(ns, N, K, device="cuda")

        def atomic(tile):
            return lambda: ext.gemm(dy, False, x, False, out, N, K, T, 3, None, None, None, 0, None, 0, 0, 0, None, 0,
                                    0.0, ks, tile, None, None)

        def store_reduce():
            ext.gemm(dy, False, x, False, ws, N, K, T, 4, None, None, None, 0, None, 0, 0, 0, None, 0, 0.0, ks, 14,
                     None, None)
            ext.splitk_reduce(ws, ns, out, True)

        res = {}
        for lbl, f in (("t12 atomic", atomic(12)), ("t14 atomic", atomic(14)), ("t14 store", store_reduce)):
            out.zero_()
            f()
            torch.cuda.synchronize()
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            res[lbl] = (timeit(f), err)
        line = " | ".join(f"{k} {v[0]:.3f} ms (err {v[1]:.1e})" for k, v in res.items())
        print(f"wgrad {name} N{N} K{K} splits {ns:3d}: {line}", flush=True)
