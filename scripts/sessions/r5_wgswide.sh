#!/bin/bash
# Round 5: weight-gradient width for the wide weights (256 in-tree vs 384 / 512, ab_wwNNN/) on
# ViT-H/14 fp8 b256 and ViT-L/16-384 b128.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5wgswide}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log")"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  step 300 h14_256_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 3
  for w in 384 512; do PVR_PKG_ROOT=$R/ab_ww$w step 300 h14_${w}_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 3; done
  step 300 l16_256_$i.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 8 --warmup 3
  for w in 384 512; do PVR_PKG_ROOT=$R/ab_ww$w step 300 l16_${w}_$i.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 8 --warmup 3; done
done
