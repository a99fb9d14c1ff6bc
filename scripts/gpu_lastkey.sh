#!/bin/bash
# N = 256 + 1 attention backward (main kernel over 256 keys + last-key streaming kernel): checks,
# kernel times at ViT-H/14 shapes with the split on / off, the H/14 bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/lastkey
timeout -k 10 200 python -u tests/kernel_checks.py > gpurun_out/lastkey/checks.log 2>&1; rc=$?
grep -i "attn_bwd.*N257\|failing" gpurun_out/lastkey/checks.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do PVR_ATTN_BWD_TAIL=$v timeout -k 10 100 python scripts/attn_shape_probe.py 2>&1 | grep B128 || exit 1; done
PVR_ATTN_BWD_TAIL=1 timeout -k 10 100 python scripts/attn_shape_probe.py 128 257 16 64 2>&1 | grep B128 || exit 1
for v in 1 0; do
  PVR_ATTN_BWD_TAIL=$v timeout -k 10 300 python bench.py --model vit_h14 --batch 128 --steps 6 --warmup 2 > gpurun_out/lastkey/h14_$v.log 2>&1
  rc=$?; echo "h14 tail=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/lastkey/h14_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
