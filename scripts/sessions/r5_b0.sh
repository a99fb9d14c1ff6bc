#!/bin/bash
# Round 5: ping-pong GEMM reading the next K-tile's B0 fragments in phase (1,0) (k-contiguous B;
# ab_b0/) vs the in-tree build: kernel checks on the variant, the step's GEMMs alternating
# (gemm_ab.py), then whole-step benches alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5b0}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
PVR_PKG_ROOT=$R/ab_b0 step 600 kernels_b0.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 300 gemm_base_$i.log python scripts/gemm_ab.py
  PVR_PKG_ROOT=$R/ab_b0 step 300 gemm_b0_$i.log python scripts/gemm_ab.py
done
for i in 1 2; do
  step 200 b16_base_$i.log python bench.py
  PVR_PKG_ROOT=$R/ab_b0 step 200 b16_b0_$i.log python bench.py
done
