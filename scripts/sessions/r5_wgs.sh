#!/bin/bash
# Round 5: weight-gradient split-K width (workgroups per wgrad GEMM: 256 in-tree vs 128 / 192 / 384 /
# 512, ab_wNNN/ copies with the same .so), ViT-B/16 b256 step, alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5wgs}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log")"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2 3; do
  step 200 b16_256_$i.log python bench.py
  for w in 64 96 128 160; do PVR_PKG_ROOT=$R/ab_w$w step 200 b16_${w}_$i.log python bench.py; done
done
