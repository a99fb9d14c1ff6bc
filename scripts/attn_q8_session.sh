#!/bin/bash
# GPU session: attention forward output staging A/B (+ attention kernel checks)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-aq8}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernel_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
step 200 attn_q8.log python scripts/attn_q8_probe.py
grep -v amdgpu.ids "$O/attn_q8.log"
