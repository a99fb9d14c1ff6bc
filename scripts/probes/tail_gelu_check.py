"""Probe: split-K tail vs one-workgroup-per-tile GELU+dropout GEMM (tile 12), flipped-mask details."""
import os, sys, torch
sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or "/root/repo")
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import kernel_checks as KC
from pytorch_vit_paper_replication_amd.ops import gemm as G
M, N, K = 50432, 3072, 3072
for sd in (37, 36):
    torch.manual_seed(sd)
    seed = torch.tensor([4242], dtype=torch.int64, device="cuda")
    x, w, b = KC.bf(KC.rnd(M, K)), KC.bf(KC.rnd(N, K, scale=0.05)), KC.rnd(N)
    def run():
        u = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        h = G.linear_fwd(x, w, b, gelu_aux=u, drop=(seed, 9 << 32, 0.1))
        return h, u
    old, G.DGRAD_TAIL_UNITS = G.DGRAD_TAIL_UNITS, 0
    with KC.tile(12):
        with KC.gemm_tail(False):
            base = run()
        a = run()
    G.DGRAD_TAIL_UNITS = old
    flip = (a[0] == 0) != (base[0] == 0)
    big = flip & (torch.maximum(a[0].float().abs(), base[0].float().abs()) > 1e-20)
    idx = big.nonzero()[:8].tolist()
    print(sd, "flips", int(flip.sum()), "big", int(big.sum()), flush=True)
    for r, c in idx:
        print("  ", r, c, float(a[0][r, c]), float(base[0][r, c]), float(a[1][r, c]), float(base[1][r, c]), flush=True)
