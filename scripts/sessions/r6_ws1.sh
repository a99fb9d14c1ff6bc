#!/bin/bash
# Round 6: first run of the wave-specialized GEMM (tile 15, csrc/gemm_ws.hip) + the A0 read-ahead A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-ws1}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
timeout -k 10 600 python -u scripts/run_checks.py check_gemm > "$O/checks.log" 2>&1; rc=$?; echo "checks rc=$rc"
[ $rc -le 1 ] || exit $rc  # 1 = a check failed (numbers in the log); anything else: stop
grep -c "^ok" "$O/checks.log"; grep "^FAIL" "$O/checks.log" | head
ONLY="qkv fwd,out fwd,fc1 fwd,fc2 fwd,fc2 dgrad,fc1 dgrad,out dgrad,qkv dgrad"
run 400 gemm_ws_ab.log python scripts/gemm_ab.py --ab tiles:def,15 --only "$ONLY"
cat "$O/gemm_ws_ab.log" | grep ours
for r in 1 2; do
  run 300 gemm_main_$r.log python scripts/gemm_ab.py --only "$ONLY"
  PVR_PKG_ROOT=abv/nopre run 300 gemm_nopre_$r.log python scripts/gemm_ab.py --only "$ONLY"
done
for r in 1 2; do
  run 200 b16_main_$r.log python bench.py
  PVR_PKG_ROOT=abv/nopre run 200 b16_nopre_$r.log python bench.py
  PVR_GEMM_WS=gelu,dgelu run 200 b16_ws_$r.log python bench.py
done
