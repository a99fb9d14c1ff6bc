#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/fp8_debug.py > gpurun_out/dbg.log 2>&1; echo rc=$?; cat gpurun_out/dbg.log
