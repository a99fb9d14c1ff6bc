#!/bin/bash
# Pipelined attention backward: GPU numerics, then A/B microbench: 8-wave vs 4-wave pipelined kernel
# vs the two-kernel backward.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/pipe; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pipe/pytest.log; [ $rc -ne 0 ] && exit $rc
PVR_ATTN_BWD_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe/pytest4.log 2>&1
rc=$?; tail -1 gpurun_out/pipe/pytest4.log; [ $rc -ne 0 ] && exit $rc
for v in 8 4 x 8 4 x; do
  if [ "$v" = x ]; then E="PVR_ATTN_BWD_PIPE=0"; else E="PVR_ATTN_BWD_WAVES=$v"; fi
  env $E timeout -k 10 120 python scripts/bench_kernels.py --only attn > gpurun_out/pipe/kb_$v.log 2>&1 || exit $?
  echo "$E $(grep attn_bwd gpurun_out/pipe/kb_$v.log | tr '\n' ' ')"
done
exit 0
