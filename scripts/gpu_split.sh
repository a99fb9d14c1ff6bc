#!/bin/bash
# Split-store persistent GEMM epilogue: kernel checks, epilogue microbenchmarks with the split on/off,
# headline bench A/B (same box, alternating).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/split
timeout -k 10 200 python -u tests/kernel_checks.py > gpurun_out/split/checks.log 2>&1; rc=$?
grep -i "t13\|13)\|failing\|BAD\|FAIL" gpurun_out/split/checks.log | head -12; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  PVR_PPP_SPLIT=$v timeout -k 10 200 python scripts/bench_kernels.py --only epi > gpurun_out/split/epi$v.log 2>&1; rc=$?
  echo "PVR_PPP_SPLIT=$v"; grep "tile13\|GELU+drop" gpurun_out/split/epi$v.log; [ $rc -ne 0 ] && exit $rc
done
for i in 1 2; do
  for v in 1 0; do
    PVR_PPP_SPLIT=$v timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/split/b$v$i.log 2>&1
    rc=$?; echo "split=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/split/b$v$i.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
