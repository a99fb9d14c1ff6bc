#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tests/kernel_checks.py > gpurun_out/checks.log 2>&1; rc=$?; grep -v "^OK" gpurun_out/checks.log | tail -5; echo "checks rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh
