#!/bin/bash
# Round 6 A/B session: kernel checks on the main tree, then GEMM timings (scripts/gemm_ab.py) and the
# headline bench alternating between the main tree and the A/B tree(s) given as arguments
# (scripts/mk_abtree.sh builds them).   gpurun -- bash scripts/sessions/r6_ab.sh <tag> <checks> abv/x [abv/y ...]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
TAG=$1; CHECKS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 20 "$O/$log"; exit $rc; }; }
if [ "$CHECKS" != "-" ]; then run 600 checks.log python -u scripts/run_checks.py "$CHECKS"; grep -c "^ok" "$O/checks.log"; fi
for r in 1 2; do
  run 300 gemm_main_$r.log python scripts/gemm_ab.py
  for v in "$@"; do n=$(basename $v); PVR_PKG_ROOT=$v run 300 gemm_${n}_$r.log python scripts/gemm_ab.py; done
done
for r in 1 2 3; do
  run 200 b16_main_$r.log python bench.py
  for v in "$@"; do n=$(basename $v); PVR_PKG_ROOT=$v run 200 b16_${n}_$r.log python bench.py; done
done
