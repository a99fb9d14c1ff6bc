#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
PVR_DEBUG_KERNELS=1 timeout -k 10 400 python tests/kernel_checks.py > gpurun_out/checks_debug.log 2>&1; rc=$?; grep -v "^OK" gpurun_out/checks_debug.log | tail -5; echo "debug-kernel checks rc=$rc"
