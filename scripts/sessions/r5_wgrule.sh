#!/bin/bash
# Round 5: narrow-weight wgrad width rule (in-tree) vs the previous commit (ab_prev/, same .so):
# GPU suite on the new tree, ViT-B/16 b256 (3 pairs), ViT-H/14 fp8 (1 pair) alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5wgrule}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed' "$O/$log" | tail -1)"; [ $rc -eq 0 ] || exit $rc; }
step 1100 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for i in 1 2 3; do
  PVR_PKG_ROOT=$R/ab_prev step 200 b16_prev_$i.log python bench.py
  step 200 b16_new_$i.log python bench.py
done
PVR_PKG_ROOT=$R/ab_prev step 300 h14_prev.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
step 300 h14_new.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
