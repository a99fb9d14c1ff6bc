#!/bin/bash
# Round 5: attention backward with LDS reads a group ahead (NW template): kernel checks, new vs HEAD~
# (ab_old/) backward times alternating, phase stamps (ab_st/).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5attn4}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "bwd\|passed\|failed\|total\|sum of" "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 200 ab_new_$i.log python scripts/attn_ab.py --bwd --rounds 3
  PVR_PKG_ROOT=$R/ab_old step 200 ab_old_$i.log python scripts/attn_ab.py --bwd --rounds 3
done
PVR_PKG_ROOT=$R/ab_st step 200 stamps.log python scripts/attn_stamps.py
