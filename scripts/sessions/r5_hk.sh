#!/bin/bash
# Round 5: dropout bits hashed inside the persistent GEMM's K loop (MFMA issue gaps) instead of in
# the epilogue (in-tree build) vs the committed kernel (ab_head/): kernel checks, the step's GEMMs
# alternating (gemm_ab.py), then whole-step benches alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5hk}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels_hk.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 300 gemm_base_$i.log python scripts/gemm_ab.py
  step 300 gemm_hk_$i.log python scripts/gemm_ab.py
done
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 200 b16_base_$i.log python bench.py
  step 200 b16_hk_$i.log python bench.py
done
