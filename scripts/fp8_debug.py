import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests import kernel_checks as KC
for (M, N, K, r) in [(700, 2304, 768, False), (700, 2304, 768, True), (591, 2304, 768, True), (700, 768, 768, True),
                     (3000, 768, 1280, True), (512, 256, 128, True), (256, 256, 128, True), (256, 256, 128, False)]:
    torch.manual_seed(0)
    name, err, tol = KC.check_gemm_fp8(M, N, K, r, False)
    print(f"{name:70s} err={err:.3e}", flush=True)
