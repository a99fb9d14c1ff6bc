#!/bin/bash
# Round 5: tile rule (persistent kernel for K <= 2048 only, dGELU dgrad persistent; in-tree ops/gemm.py)
# vs the round-4 rule (ab_head/, same .so) on the ViT-L/16-384 b128 step, alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5l16rule}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "images/sec\|passed" "$O/$log" | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
step 400 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 300 l16_base_$i.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 10 --warmup 3
  step 300 l16_new_$i.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 10 --warmup 3
done
