#!/bin/bash
# Round 5, timing-only probe of the LDS-bound hypothesis: the ping-pong K loops with the B1 fragment
# reads skipped (ab_sb1/: 4 of 24 reads per K-tile) or the A1 reads skipped (ab_sa1/: 8 of 24), wrong
# results, vs the in-tree kernels: the step's GEMMs alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5lds}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  step 300 gemm_base_$i.log python scripts/gemm_ab.py
  PVR_PKG_ROOT=$R/ab_sb1 step 300 gemm_sb1_$i.log python scripts/gemm_ab.py
  PVR_PKG_ROOT=$R/ab_sa1 step 300 gemm_sa1_$i.log python scripts/gemm_ab.py
done
