#!/bin/bash
# GPU session: fp8 epilogues without the unused bf16 packing (c_skip) - checks, epilogue probe, H/14 bench
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-cskip}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernel_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
step 300 probe_h14.log python scripts/fc1_epi_probe.py --model h14
grep -v amdgpu.ids "$O/probe_h14.log"
step 300 h14_a.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
step 300 h14_b.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
