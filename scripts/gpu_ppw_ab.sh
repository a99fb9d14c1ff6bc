#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tests/kernel_checks.py > gpurun_out/checks.log 2>&1 || { tail -5 gpurun_out/checks.log; exit 1; }
tail -1 gpurun_out/checks.log
for ppw in 12 1 2 3 6; do
  PVR_ATTN_BWD_PPW=$ppw timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_ppw$ppw.log 2>&1 || exit $?
  echo "ppw $ppw: $(grep -o '"value": [0-9.]*' gpurun_out/bench_ppw$ppw.log)"
done
for ppw in 12 1 3; do
  PVR_ATTN_BWD_PPW=$ppw timeout -k 10 100 python scripts/bench_kernels.py --only attn > gpurun_out/kb_ppw$ppw.log 2>&1 || exit $?
  echo "ppw $ppw: $(grep attn_bwd gpurun_out/kb_ppw$ppw.log)"
done
