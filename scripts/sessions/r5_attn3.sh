#!/bin/bash
# Round 5: attention backward A/B (S/dP one block ahead vs at the top of its block vs HEAD~ kernel)
# and phase stamps of both orders (diagnostic builds ab_st / ab_stnp).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5attn3}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "bwd\|cyc\|total\|sum" "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  step 200 ab_pipe_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
  PVR_PKG_ROOT=$R/ab_np step 200 ab_np_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
  PVR_PKG_ROOT=$R/ab_old step 200 ab_old_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
done
PVR_PKG_ROOT=$R/ab_st step 200 stamps_pipe.log python scripts/attn_stamps.py
PVR_PKG_ROOT=$R/ab_stnp step 200 stamps_nopipe.log python scripts/attn_stamps.py
