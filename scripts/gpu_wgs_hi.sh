#!/bin/bash
# Weight-gradient split count above one workgroup per CU (shorter-lived side-stream workgroups give
# the high-priority dgrad chain CUs sooner, at the cost of more split-K partial traffic); also the
# packed-GELU build's fc1 epilogue microbenchmark.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/wgs
timeout -k 10 120 python -u tests/kernel_checks.py > gpurun_out/wgs/checks.log 2>&1; rc=$?
grep -i "gelu\|failing" gpurun_out/wgs/checks.log | head -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/bench_kernels.py --only epi > gpurun_out/wgs/epi.log 2>&1; grep "fc1 fwd" gpurun_out/wgs/epi.log
for i in 1 2; do
  for w in 256 512 384; do
    PVR_WGRAD_WGS=$w timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/wgs/w$w.log 2>&1
    rc=$?; echo "wgs=$w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/wgs/w$w.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
