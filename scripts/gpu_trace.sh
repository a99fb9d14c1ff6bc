#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace" -o step --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/trace.log" 2>&1
echo rc=$?
