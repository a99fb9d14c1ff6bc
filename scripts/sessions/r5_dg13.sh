#!/bin/bash
# Round 5: dGELU dgrad on the persistent kernel (tile 13, in-tree ops/gemm.py) vs the one-tile kernel
# (ab_head/: same .so, round-4 rule): checks, the step's GEMMs and the whole step alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5dg13}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "images/sec\|passed" "$O/$log" | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
step 400 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 300 gemm_base_$i.log python scripts/gemm_ab.py
  step 300 gemm_dg13_$i.log python scripts/gemm_ab.py
done
for i in 1 2 3; do
  PVR_PKG_ROOT=$R/ab_head step 200 b16_base_$i.log python bench.py
  step 200 b16_dg13_$i.log python bench.py
done
PVR_PKG_ROOT=$R/ab_head step 300 h14_base.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
step 300 h14_dg13.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
