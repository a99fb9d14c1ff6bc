#!/bin/bash
# Pipelined attention backward: GPU numerics, then A/B microbench vs the two-kernel backward.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/pipe; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pipe/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  PVR_ATTN_BWD_PIPE=$v timeout -k 10 120 python scripts/bench_kernels.py --only attn > gpurun_out/pipe/kb_$v.log 2>&1 || exit $?
  echo "pipe=$v $(grep attn_bwd gpurun_out/pipe/kb_$v.log)"
done
exit 0
