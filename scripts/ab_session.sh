#!/bin/bash
# A/B session (round 4): bench variants interleaved, GEMM table vs hipBLASLt, peak memory.
# Every GPU step under its own timeout; the first failure ends it.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 300 tail_check.log python -u scripts/tail_check.py
for r in 1 2; do
  step 200 b_off_$r.log python bench.py --no-gemm-tail
  step 200 b_on_$r.log python bench.py
  step 200 b_ser_on_$r.log python bench.py --serial-wgrad
  step 200 b_ser_off_$r.log python bench.py --serial-wgrad --no-gemm-tail
  step 200 b_w8_$r.log python bench.py --no-gemm-tail --side-window 8
  step 200 b_w0_$r.log python bench.py --no-gemm-tail --side-window 0
done
step 300 h14_w0.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4 --side-window 0
step 300 h14_w4.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4 --side-window 4
step 300 h14_w8.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4 --side-window 8
step 500 gemm_ab_tail.log python -u scripts/gemm_ab.py --ab tail --rounds 4
