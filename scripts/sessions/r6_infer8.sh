#!/bin/bash
# Round 6: fp8 serving (no GELU derivative, e4m3 copies only under inference_mode): kernel checks,
# then bench.py --infer bf16 vs fp8 at ViT-B/16 and ViT-H/14.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-infer8}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 300 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider
grep "fp8 inference" "$O/kernels.log" | cut -c1-250
for i in 1 2; do
  run 240 b16_bf16_$i.log python bench.py --infer --steps 30 --warmup 5
  run 240 b16_fp8_$i.log python bench.py --infer --dtype fp8 --steps 30 --warmup 5
done
run 240 b16_bf16_b1024.log python bench.py --infer --batch 1024 --steps 20 --warmup 5
run 240 b16_fp8_b1024.log python bench.py --infer --dtype fp8 --batch 1024 --steps 20 --warmup 5
for i in 1 2; do
  run 300 h14_bf16_$i.log python bench.py --infer --model vit_h14 --steps 10 --warmup 3
  run 300 h14_fp8_$i.log python bench.py --infer --model vit_h14 --dtype fp8 --steps 10 --warmup 3
done
