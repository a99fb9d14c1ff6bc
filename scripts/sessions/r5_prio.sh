#!/bin/bash
# Round 5: ping-pong GEMM wave priority: per-phase s_setprio 1 around the MFMA block (in-tree) vs none
# (ab_p1/, -DPVR_PP_PRIO=1) vs static priority 1 for waves 4-7 (ab_p2/, =2): GEMM checks on the
# variants, the step's GEMMs and the whole step alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5prio}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
for v in p1 p2; do
  PVR_PKG_ROOT=$R/ab_$v step 400 kernels_$v.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
done
for i in 1 2; do
  step 300 gemm_base_$i.log python scripts/gemm_ab.py
  PVR_PKG_ROOT=$R/ab_p1 step 300 gemm_p1_$i.log python scripts/gemm_ab.py
  PVR_PKG_ROOT=$R/ab_p2 step 300 gemm_p2_$i.log python scripts/gemm_ab.py
done
for i in 1 2; do
  step 200 b16_base_$i.log python bench.py
  PVR_PKG_ROOT=$R/ab_p1 step 200 b16_p1_$i.log python bench.py
  PVR_PKG_ROOT=$R/ab_p2 step 200 b16_p2_$i.log python bench.py
done
