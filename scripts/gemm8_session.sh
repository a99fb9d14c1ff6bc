#!/bin/bash
# GPU session: fp8 persistent dGELU dgrad A/B (mode 1 vs 3) - kernel checks, epilogue probe, H/14 benches
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-g8}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernel_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
for m in 1 3; do
  step 300 probe_p$m.log python scripts/fc1_epi_probe.py --model h14 --persistent $m
  grep -v amdgpu.ids "$O/probe_p$m.log"
done
for m in 1 3 1 3; do
  step 300 h14_p$m.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4 --fp8-persistent $m
done
