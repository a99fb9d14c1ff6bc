#!/bin/bash
# Persistent GEMM (tile 13) store-overlap A/B: GPU kernel checks with and without, then the fused
# epilogue microbenchmarks (tile 12 vs 13 per epilogue kind) alternating PVR_PPP_OVERLAP=1/0.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ppp; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ppp/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ppp/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 1 0; do
    PVR_PPP_OVERLAP=$v timeout -k 10 200 python scripts/bench_kernels.py --only epi > gpurun_out/ppp/epi_$v.log 2>&1 || exit $?
    echo "== PVR_PPP_OVERLAP=$v"; grep -E "tile1[23]|GELU tile13|bias\+GELU" gpurun_out/ppp/epi_$v.log
  done
done
exit 0
