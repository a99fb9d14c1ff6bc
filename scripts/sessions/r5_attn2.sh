#!/bin/bash
# Round 5: attention backward, S / dP one block ahead (3-slot ring, NW template): kernel checks, then
# old (ab_old/, HEAD build) vs new backward times at the BASELINE shapes, alternating, then in-step.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5attn2}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 3 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 900 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 200 ab_new_$i.log python scripts/attn_ab.py --bwd --rounds 3
  PVR_PKG_ROOT=$R/ab_old step 200 ab_old_$i.log python scripts/attn_ab.py --bwd --rounds 3
done
step 300 l16.log python bench.py --model vit_l16 --image-size 384 --steps 6 --warmup 3
step 300 h14.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
step 200 b16.log python bench.py
