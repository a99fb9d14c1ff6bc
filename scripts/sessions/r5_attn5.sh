#!/bin/bash
# Round 5: attention backward read-ahead experiments on the round-4 kernel (macro builds ab_tr / ab_dq /
# ab_trdq vs the in-tree build), alternating; phase stamps of the base and of both read-aheads.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5attn5}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "bwd l16\|bwd h14\|passed\|failed\|total\|sum of" "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  step 200 ab_base_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
  for v in tr dq trdq; do PVR_PKG_ROOT=$R/ab_$v step 200 ab_${v}_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14; done
done
PVR_PKG_ROOT=$R/ab_st step 200 stamps_base.log python scripts/attn_stamps.py
PVR_PKG_ROOT=$R/ab_sttrdq step 200 stamps_trdq.log python scripts/attn_stamps.py
PVR_PKG_ROOT=$R/ab_trdq step 600 kernels_trdq.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
