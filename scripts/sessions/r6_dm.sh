#!/bin/bash
# Round 6: dropout keep-masks from LN2 read by the fc1 / fc2 epilogues: checks, GEMM timings, the
# headline bench alternating PVR_DROP_MASK=1 / 0.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-dm1}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 300 checks.log python -u scripts/run_checks.py check_drop_masks,check_gemm_gelu,check_gemm_dropout,check_ln
cat "$O/checks.log" | grep -v amdgpu.ids
for r in 1 2 3; do
  run 240 on_$r.log python bench.py --steps 30 --warmup 5
  PVR_DROP_MASK=0 run 240 off_$r.log python bench.py --steps 30 --warmup 5
done
