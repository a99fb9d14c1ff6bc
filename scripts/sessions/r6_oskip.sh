#!/bin/bash
# Round 6: fp8 serving with the e4m3-only attention output (bf16 O not stored under inference):
# kernel checks, then A/B against abv/pre_o (the tree before it), alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-oskip}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 300 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider
grep "fp8 inference" "$O/kernels.log" | cut -c1-250
for i in 1 2 3; do
  PVR_PKG_ROOT=abv/pre_o run 300 h14_pre_$i.log python bench.py --infer --model vit_h14 --dtype fp8 --steps 10 --warmup 3
  run 300 h14_new_$i.log python bench.py --infer --model vit_h14 --dtype fp8 --steps 10 --warmup 3
  PVR_PKG_ROOT=abv/pre_o run 240 b16_pre_$i.log python bench.py --infer --dtype fp8 --steps 30 --warmup 5
  run 240 b16_new_$i.log python bench.py --infer --dtype fp8 --steps 30 --warmup 5
done
