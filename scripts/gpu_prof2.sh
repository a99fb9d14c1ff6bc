#!/bin/bash
# rocprofv3 kernel stats of the current fused step (B/16 b256)
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/prof3"
export TMPDIR=/tmp
cd /tmp
PVR_SIDE_WGRAD=${PVR_SIDE_WGRAD:-1} timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof3" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof3.log" 2>&1
echo rc=$?
