#!/bin/bash
# Full training step under rocprofv3 --kernel-trace --stats (per-kernel time per step).
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out/prof2"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof2" -o step --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof2/run.log" 2>&1
rc=$?; echo "rc=$rc"; grep metric "$R/gpurun_out/prof2/run.log"; exit $rc
