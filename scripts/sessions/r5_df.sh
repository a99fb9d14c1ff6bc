#!/bin/bash
# Round 5: ping-pong K loops issuing each phase's LDS-DMA before its fragment reads (ab_df/) vs after
# them (in-tree): kernel checks on the variant, the step's GEMMs and the whole step alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5df}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
PVR_PKG_ROOT=$R/ab_df step 600 kernels_df.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 300 gemm_base_$i.log python scripts/gemm_ab.py
  PVR_PKG_ROOT=$R/ab_df step 300 gemm_df_$i.log python scripts/gemm_ab.py
done
for i in 1 2; do
  step 200 b16_base_$i.log python bench.py
  PVR_PKG_ROOT=$R/ab_df step 200 b16_df_$i.log python bench.py
done
