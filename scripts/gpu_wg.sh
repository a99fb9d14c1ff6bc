#!/bin/bash
# wgrad store-and-reduce session: variant probe, kernel numerics, bench A/B (PVR_WGRAD_REDUCE 1 vs 0)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/wgrad_probe.py > gpurun_out/wgrad_probe.log 2>&1 || { echo probe rc=$?; tail -20 gpurun_out/wgrad_probe.log; exit 1; }
cat gpurun_out/wgrad_probe.log
timeout -k 10 600 python tests/kernel_checks.py > gpurun_out/kchk.log 2>&1 || { echo kchk rc=$?; tail -30 gpurun_out/kchk.log; exit 1; }
tail -3 gpurun_out/kchk.log
AB_VAR=PVR_WGRAD_REDUCE AB_A=1 AB_B=0 bash scripts/gpu_ab.sh
