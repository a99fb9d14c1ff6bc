#!/bin/bash
# Attention backward body/tail split (N = 257 / 577): kernel checks, then ViT-H/14 and ViT-L/16@384
# benches with the split on / off (same box).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/atail
timeout -k 10 200 python -u tests/kernel_checks.py > gpurun_out/atail/checks.log 2>&1; rc=$?
grep -i "attn_bwd\|failing" gpurun_out/atail/checks.log | head -20; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  PVR_ATTN_BWD_TAIL=$v timeout -k 10 300 python bench.py --model vit_h14 --batch 128 --steps 6 --warmup 2 > gpurun_out/atail/h14_$v.log 2>&1
  rc=$?; echo "h14 tail=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/atail/h14_$v.log)"; [ $rc -ne 0 ] && exit $rc
  PVR_ATTN_BWD_TAIL=$v timeout -k 10 300 python bench.py --model vit_l16 --image-size 384 --batch 64 --steps 6 --warmup 2 > gpurun_out/atail/l16_$v.log 2>&1
  rc=$?; echo "l16@384 tail=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/atail/l16_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
