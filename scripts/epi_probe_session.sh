#!/bin/bash
# GPU session: kernel checks, fc1 / dGELU epilogue probes, BASELINE benches (round 4)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-probe}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernel_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
step 200 probe_h14.log python scripts/fc1_epi_probe.py --model h14
step 200 probe_b16.log python scripts/fc1_epi_probe.py --model b16
cat "$O/probe_h14.log" "$O/probe_b16.log" | grep -v amdgpu.ids
step 300 tail_kt.log python scripts/tail_kt_ab.py
cat "$O/tail_kt.log" | grep -v amdgpu.ids
step 300 h14_def.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
step 200 b_def.log python bench.py
