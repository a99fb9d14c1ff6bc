#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for cap in 2048 1024 512 256; do
  PVR_LN_BWD_BLOCKS=$cap timeout -k 10 120 python scripts/bench_kernels.py --only ln > gpurun_out/kb_ln_$cap.log 2>&1 || exit $?
  echo "cap $cap"; grep -v amdgpu gpurun_out/kb_ln_$cap.log
done
