#!/bin/bash
# Round 5: weight-gradient split-K width 144 (ab_w144/) vs 256 (in-tree) on ViT-L/16-384 b128.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5wgs4}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log")"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  step 300 l16_256_$i.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 10 --warmup 3
  PVR_PKG_ROOT=$R/ab_w144 step 300 l16_144_$i.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 10 --warmup 3
done
