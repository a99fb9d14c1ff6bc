#!/bin/bash
# Round 5 timing experiment: GEMM bias epilogue stores as 8 rows x 128 B per instruction (wrong data
# placement, timing only: ab_exp build with -DPVR_EXP_FULLLINE) vs 16 rows x 64 B (in-tree build)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5g; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 120 python -u scripts/gemm_stamps.py --epi bias --tiles 256,2304 > $O/base_$r.log 2>&1 || exit 1
  PVR_PKG_ROOT=$R/ab_exp timeout -k 10 120 python -u scripts/gemm_stamps.py --epi bias --tiles 256,2304 > $O/full_$r.log 2>&1 || exit 1
done
tail -n 2 $O/*.log
