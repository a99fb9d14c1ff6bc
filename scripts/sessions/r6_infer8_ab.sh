#!/bin/bash
# Round 6: fp8 serving A/B, this tree vs abv/pre_infer (the tree before the inference-only fp8 epilogue /
# copy skips), alternating, ViT-B/16 b256 and ViT-H/14 b256.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-infer8_ab}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
for i in 1 2; do
  PVR_PKG_ROOT=abv/pre_infer run 240 b16_pre_$i.log python bench.py --infer --dtype fp8 --steps 30 --warmup 5
  run 240 b16_new_$i.log python bench.py --infer --dtype fp8 --steps 30 --warmup 5
  PVR_PKG_ROOT=abv/pre_infer run 300 h14_pre_$i.log python bench.py --infer --model vit_h14 --dtype fp8 --steps 10 --warmup 3
  run 300 h14_new_$i.log python bench.py --infer --model vit_h14 --dtype fp8 --steps 10 --warmup 3
done
