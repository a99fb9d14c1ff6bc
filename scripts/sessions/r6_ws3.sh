#!/bin/bash
# Round 6: tile-15 cache-policy A/B (abv/nt1: nt u stores + nt epilogue stores; nt2: + sc1|nt scratch
# loads; nt3: nt u stores with the barrier-only epilogue; abv/abl1: plain u stores, barrier-only epilogue)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-ws6}; mkdir -p "$O"; shift
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc"; grep " ours " "$O/$log" | cut -c1-100; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
ONLY="fc1 fwd   bias+GELU+drop+aux,fc1 dgrad,fc2 dgrad dGELU+colsum,qkv fwd"
[ -n "$SKIPMAIN" ] || run 300 main.log python scripts/gemm_ab.py --ab tiles:def,15 --only "$ONLY" --rounds 2
for a in "$@"; do PVR_PKG_ROOT=abv/$a run 300 $a.log python scripts/gemm_ab.py --ab tiles:15 --only "$ONLY" --rounds 2; done
