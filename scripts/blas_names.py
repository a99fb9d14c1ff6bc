"""Run hipBLASLt (torch.matmul) on the ViT-B/16 GEMM shapes so rocprofv3 records its kernel choices."""
import torch

T = 50432
for n, k in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(x, w.t())
    torch.cuda.synchronize()
    print("shape", n, k, flush=True)
