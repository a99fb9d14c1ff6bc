#!/bin/bash
# Round 5: attention backward (generic + persistent whole-head kernels) with static priority 1 for the
# second wave of each SIMD (ab_ap/, -DPVR_ATTN_PRIO) vs none (in-tree): checks, backward times and the
# ViT-B/16 step alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5aprio}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "attn bwd\|passed\|failed\|images/sec" "$O/$log" | cut -c1-140; [ $rc -eq 0 ] || exit $rc; }
PVR_PKG_ROOT=$R/ab_ap step 400 kernels_ap.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 200 attn_base_$i.log python scripts/attn_ab.py --bwd --rounds 3
  PVR_PKG_ROOT=$R/ab_ap step 200 attn_ap_$i.log python scripts/attn_ab.py --bwd --rounds 3
done
for i in 1 2; do
  step 200 b16_base_$i.log python bench.py
  PVR_PKG_ROOT=$R/ab_ap step 200 b16_ap_$i.log python bench.py
done
