#!/bin/bash
# Round 6: tile 15 with the LDS hand-off: GEMM kernel checks, then tile 15 vs the defaults and the
# ablations (abv/abl1: barrier-only epilogue waves; abv/abl3: no hand-off, MFMA waves alone).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-ws7}; mkdir -p "$O"; shift
if [ -z "$SKIPCHECK" ]; then
  timeout -k 10 600 python -u scripts/run_checks.py check_gemm > "$O/checks.log" 2>&1; rc=$?; echo "checks rc=$rc"
  grep -c "^ok" "$O/checks.log"; grep "^FAIL" "$O/checks.log" | head
  [ $rc -le 1 ] || exit $rc
fi
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc"; grep " ours " "$O/$log" | cut -c1-100; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
ONLY=${ONLY:-"qkv fwd,out fwd,fc1 fwd   bias+GELU+drop+aux,fc2 fwd,fc2 dgrad dGELU+colsum,fc1 dgrad,out dgrad,qkv dgrad"}
run 400 main.log python scripts/gemm_ab.py --ab tiles:def,15 --only "$ONLY" --rounds 2
for a in "$@"; do PVR_PKG_ROOT=abv/$a run 300 $a.log python scripts/gemm_ab.py --ab tiles:15 --only "$ONLY" --rounds 2; done
