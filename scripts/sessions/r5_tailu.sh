#!/bin/bash
# Round 5: dgrad split-K tail limit (DGRAD_TAIL_UNITS 64 in-tree vs 0 = unlimited / 128 / 32,
# ab_tuNN/ copies, same .so) and stream priority (--main-prio 0) with the narrower weight gradients.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5tailu}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log")"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2 3; do
  step 200 b16_64_$i.log python bench.py
  for u in 0 128 32; do PVR_PKG_ROOT=$R/ab_tu$u step 200 b16_${u}_$i.log python bench.py; done
  step 200 b16_prio0_$i.log python bench.py --main-prio 0
done
