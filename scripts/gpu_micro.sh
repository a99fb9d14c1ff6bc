#!/bin/bash
# Two-stream micro-batched encoder blocks: numerics checks, then the headline bench A/B
# (PVR_MICRO=2 default vs PVR_MICRO=1), and the b512 per-GPU config.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/micro
timeout -k 10 200 python -u -c "
import torch, sys
sys.path.insert(0, '.')
from tests import kernel_checks as KC
for f in (KC.check_vit_micro, lambda: KC.check_vit_micro(64), KC.check_vit_block_link_micro, KC.check_vit_block_link):
    n, e, t = f(); print('OK ' if e <= t else 'BAD', n, f'{e:.3e}', t, flush=True)
" > gpurun_out/micro/checks.log 2>&1
rc=$?; cat gpurun_out/micro/checks.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
for v in "m2:2" "m1:1" "m2b:2" "m1b:1"; do
  n=${v%%:*}; m=${v#*:}
  PVR_MICRO=$m timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/micro/$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/micro/$n.log)"; [ $rc -ne 0 ] && exit $rc
done
PVR_MICRO=2 timeout -k 10 200 python bench.py --steps 8 --warmup 3 --batch 512 > gpurun_out/micro/b512.log 2>&1
rc=$?; echo "b512 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/micro/b512.log)"
exit $rc
