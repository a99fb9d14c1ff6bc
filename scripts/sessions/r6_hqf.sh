#!/bin/bash
# Round 6: whole-head attention forward with 2 query fragments per wave: checks, attn_ab timing,
# headline bench alternating with abv/hqf1 (the round-5 form, 1 fragment per wave).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-hqf}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 300 checks.log python -u scripts/run_checks.py check_attn_fwd
grep -v amdgpu.ids "$O/checks.log"
run 300 attn_ab.log python scripts/attn_ab.py --shapes b16 --ab hqf --rounds 6
grep -v amdgpu.ids "$O/attn_ab.log" | tail -n 4
for r in 1 2 3; do
  run 240 main_$r.log python bench.py --steps 30 --warmup 5
  PVR_PKG_ROOT=abv/hqf1 run 240 hqf1_$r.log python bench.py --steps 30 --warmup 5
done
