#!/bin/bash
# Round 6: tile-15 ablations (abv/abl1: epilogue waves only keep barriers; abl2: + no u stores;
# abl3: epilogue waves exit at the start) against the full kernel.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-ws2}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc"; grep " ours " "$O/$log" | cut -c1-100; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
ONLY="fc1 fwd   bias+GELU+drop+aux,fc1 dgrad,fc2 dgrad dGELU+colsum,qkv fwd"
run 300 main.log python scripts/gemm_ab.py --ab tiles:def,15 --only "$ONLY" --rounds 2
for a in 1; do PVR_PKG_ROOT=abv/abl$a run 300 abl$a.log python scripts/gemm_ab.py --ab tiles:15 --only "$ONLY" --rounds 2; done
