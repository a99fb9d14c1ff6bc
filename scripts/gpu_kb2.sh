#!/bin/bash
# kernel checks + selected microbenchmarks: ONLY=ln,attn TILES=12 bash scripts/gpu_kb2.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tests/kernel_checks.py > gpurun_out/checks.log 2>&1; rc=$?; grep -v "^OK" gpurun_out/checks.log | tail -5; echo "checks rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python scripts/bench_kernels.py --tiles ${TILES:-12} --only ${ONLY:-ln,attn} > gpurun_out/kbench4.log 2>&1; rc=$?; cat gpurun_out/kbench4.log; echo "kbench rc=$rc"
[ $rc -le 1 ] || exit $rc
[ -z "$BENCH" ] || { timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log | cut -c1-200; }
