#!/bin/bash
# Round 5: one epilogue instance per reachable epilogue (GELU / dGELU kernels carried an identical
# second copy for the residual flag: half the code) in-tree vs the committed kernel (ab_head/):
# kernel checks, the step's GEMMs alternating (gemm_ab.py), then whole-step benches alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5dd}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels_dd.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 300 gemm_base_$i.log python scripts/gemm_ab.py
  step 300 gemm_dd_$i.log python scripts/gemm_ab.py
done
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 200 b16_base_$i.log python bench.py
  step 200 b16_dd_$i.log python bench.py
done
