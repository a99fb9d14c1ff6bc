#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python ${PROBE:-scripts/wgrad_probe.py} > gpurun_out/probe.log 2>&1; echo rc=$?; cat gpurun_out/probe.log
