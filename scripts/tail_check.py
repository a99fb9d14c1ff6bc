import sys, os, torch
sys.path.insert(0, os.getcwd())
from tests import kernel_checks as K
torch.manual_seed(0)
bad = 0
for fn in [lambda: K.check_gemm_tail_split(50432, 768, 3072, "resid_drop"),
           lambda: K.check_gemm_tail_split(50432, 768, 2304, "resid_drop"),
           lambda: K.check_gemm_tail_split(50432, 3072, 3072, "gelu"),
           lambda: K.check_gemm_tail_split(50432, 3072, 3072, "dgelu"),
           lambda: K.check_gemm_tail_split(50176, 768, 3072, "patch"),
           K.check_gemm_tail_split_fp8]:
    name, m, l = fn()
    torch.cuda.synchronize()
    ok = K.passed(m, l); bad += not ok
    print(("OK  " if ok else "FAIL"), name, K.fmt_metrics(m, l), flush=True)
sys.exit(1 if bad else 0)
