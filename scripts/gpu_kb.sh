#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tests/kernel_checks.py > gpurun_out/checks.log 2>&1; rc=$?; tail -3 gpurun_out/checks.log; echo "checks rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python scripts/bench_kernels.py --tiles ${TILES:-6,9,10,11} --only gemm > gpurun_out/kbench3.log 2>&1; rc=$?; cat gpurun_out/kbench3.log; echo "kbench rc=$rc"
