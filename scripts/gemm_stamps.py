#!/usr/bin/env python3
"""In-kernel s_memtime stamps of the one-tile-per-workgroup ping-pong GEMM (tile 12): per-workgroup
prologue / main-loop / epilogue cycles, at several grid sizes, to tell a bandwidth-bound epilogue
(epilogue cycles grow with the number of workgroups storing at once) from a latency / issue-bound
one (flat).

  python scripts/gemm_stamps.py                 # qkv-fwd shape (N 2304, K 768), bias epilogue
  python scripts/gemm_stamps.py --epi gelu      # fc1 shape with the GELU + aux epilogue
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # PVR_PKG_ROOT: an A/B build
from pytorch_vit_paper_replication_amd import _ext  # noqa: E402
from pytorch_vit_paper_replication_amd.ops import gemm as G  # noqa: E402


def persistent(ext, a):
    """The persistent form (tile 13) at the ViT-B/16 b256 shape: per workgroup, K-loop and epilogue
    cycles summed over its tiles and the rest of the kernel (tile hand-offs, start, drain)."""
    T = 50432
    N, K = {"bias": (2304, 768), "resid": (768, 768), "gelu": (3072, 768), "dgelu": (3072, 768)}[a.epi]
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    out = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    seed = torch.tensor([7], dtype=torch.int64, device="cuda")
    epi, aux_, drop = (1, aux, (seed, 3 << 32, 0.1)) if a.epi == "gelu" else (0, None, (None, 0, 0.0))
    dbg = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    rows = []
    for it in range(6):
        dbg.zero_()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ext.gemm(x, True, w, True, out, T, N, K, epi, b, None, None, 0, aux_, 0, 0, 0, drop[0], drop[1], drop[2], 0, 13, dbg=dbg,
                 tail_limit=-1)
        e.record()
        torch.cuda.synchronize()
        if it >= 2:
            d = dbg.view(-1, 8).cpu().double()
            d = d[d[:, 3] > 0]
            rows.append((d, s.elapsed_time(e)))
    med = statistics.median
    for d, ms in rows[-2:]:
        nt = d[:, 3]
        total, loop, epil = d[:, 0], d[:, 1], d[:, 2]
        print(f"persistent {a.epi} M{T} N{N} K{K}: {d.shape[0]} workgroups, {ms:.3f} ms; per tile (median over workgroups): "
              f"loop {med((loop / nt).tolist()):7.0f}  epilogue {med((epil / nt).tolist()):7.0f}  other "
              f"{med(((total - loop - epil) / nt).tolist()):7.0f}  (tiles per workgroup {med(nt.tolist()):.0f}, "
              f"kernel {med(total.tolist()):.0f} cycles)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epi", default="bias", choices=["bias", "resid", "gelu", "dgelu"])
    ap.add_argument("--tiles", default="32,64,128,256,512,1024,2304")
    ap.add_argument("--persistent", action="store_true", help="the persistent form (tile 13), per-workgroup sums")
    a = ap.parse_args()
    if a.persistent:
        return persistent(_ext.ext(), a)
    ext = _ext.ext()
    N, K = {"bias": (2304, 768), "resid": (768, 768), "gelu": (3072, 768), "dgelu": (3072, 768)}[a.epi]
    ntn = N // 256
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    seed = torch.tensor([7], dtype=torch.int64, device="cuda")
    print(f"# epilogue {a.epi}, N {N}, K {K}, tile 12; cycles per workgroup (median over workgroups)", flush=True)
    for nt in [int(t) for t in a.tiles.split(",")]:
        M = max(256, (nt // ntn) * 256)
        tiles = (M // 256) * ntn
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        aux = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        dbg = torch.zeros(tiles * 8, dtype=torch.int64, device="cuda")
        args = dict(epi=0, bias=b, resid=None, aux=None, drop=(None, 0, 0.0))
        if a.epi == "resid":
            args.update(resid=r)
        elif a.epi == "gelu":
            args.update(epi=1, aux=aux, drop=(seed, 3 << 32, 0.1))
        elif a.epi == "dgelu":
            args.update(epi=2, bias=None, aux=aux)
        rows = []
        for it in range(6):
            ext.gemm(x, True, w, True, out, M, N, K, args["epi"], args["bias"], args["resid"], None, 0, args["aux"], 0, 0, 0,
                     args["drop"][0], args["drop"][1], args["drop"][2], 0, 12, dbg=dbg, tail_limit=-1)
            torch.cuda.synchronize()
            if it >= 2:
                d = dbg.view(tiles, 8).cpu().double()
                rows.append(d)
        d = torch.stack(rows).median(0).values
        pro = (d[:, 1] - d[:, 0]).tolist()
        loop = (d[:, 2] - d[:, 1]).tolist()
        epi = (d[:, 3] - d[:, 2]).tolist()
        e_row0 = (d[:, 4] - d[:, 2]).tolist()   # register-direct epilogue: row 0 (bias / inputs landed)
        e_rows = (d[:, 5] - d[:, 4]).tolist()   # rows 1-7 issued
        e_tail = (d[:, 3] - d[:, 5]).tolist()   # column sums + store drain
        med = statistics.median
        print(f"tiles {tiles:5d}: prologue {med(pro):7.0f} loop {med(loop):7.0f} epilogue {med(epi):7.0f} "
              f"(max {max(epi):7.0f}) = row0 {med(e_row0):6.0f} + rows1-7 {med(e_rows):6.0f} + tail {med(e_tail):6.0f}", flush=True)


if __name__ == "__main__":
    main()
