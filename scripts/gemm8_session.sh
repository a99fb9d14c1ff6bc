#!/bin/bash
# GPU session: fp8 persistent GEMM - kernel checks, per-GEMM A/B vs torch._scaled_mm, H/14 benches
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-g8}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernel_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
for m in 0 1 2; do
  step 300 fp8_mm_p$m.log python scripts/fp8_vs_scaled_mm.py --rounds 3 --persistent $m
  grep -v amdgpu.ids "$O/fp8_mm_p$m.log" | grep -E "fwd|dgrad"
done
for m in 0 1 2 1; do
  step 300 h14_p$m.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4 --fp8-persistent $m
done
