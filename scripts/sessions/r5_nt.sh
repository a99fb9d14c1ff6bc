#!/bin/bash
# Round 5: register-direct epilogue stores with cache-policy bits: nt (ab_nt2/, aux 2) and sc1
# (ab_nt16/, aux 16) vs none (in-tree): persistent-kernel stamps, the step's GEMMs, the whole step.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5nt}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "persistent\|images/sec\|passed" "$O/$log" | cut -c1-170; [ $rc -eq 0 ] || exit $rc; }
for v in nt2 nt16; do
  PVR_PKG_ROOT=$R/ab_$v step 400 kernels_$v.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
done
for e in bias gelu; do
  step 100 st_base_$e.log python scripts/gemm_stamps.py --persistent --epi $e
  for v in nt2 nt16; do PVR_PKG_ROOT=$R/ab_$v step 100 st_${v}_$e.log python scripts/gemm_stamps.py --persistent --epi $e; done
done
for i in 1 2; do
  step 300 gemm_base_$i.log python scripts/gemm_ab.py
  for v in nt2 nt16; do PVR_PKG_ROOT=$R/ab_$v step 300 gemm_${v}_$i.log python scripts/gemm_ab.py; done
done
for i in 1 2; do
  step 200 b16_base_$i.log python bench.py
  for v in nt2 nt16; do PVR_PKG_ROOT=$R/ab_$v step 200 b16_${v}_$i.log python bench.py; done
done
