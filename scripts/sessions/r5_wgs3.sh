#!/bin/bash
# Round 5: weight-gradient split-K width, finer (144 / 160 / 176 vs 256 in-tree) on ViT-B/16 b256,
# then 160 vs 256 on ViT-B/16 b512 and ViT-H/14 fp8 b256.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5wgs3}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log")"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2 3; do
  step 200 b16_256_$i.log python bench.py
  for w in 144 160 176; do PVR_PKG_ROOT=$R/ab_w$w step 200 b16_${w}_$i.log python bench.py; done
done
for i in 1 2; do
  step 300 b512_256_$i.log python bench.py --batch 512
  PVR_PKG_ROOT=$R/ab_w160 step 300 b512_160_$i.log python bench.py --batch 512
  step 300 h14_256_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
  PVR_PKG_ROOT=$R/ab_w160 step 300 h14_160_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
done
