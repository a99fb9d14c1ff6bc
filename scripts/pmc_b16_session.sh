#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/pmc_b16
timeout -k 10 400 bash scripts/pmc_gemm.sh pmc_b16 b16 && timeout -k 10 200 python scripts/gemm_ab.py > gpurun_out/pmc_b16/gemm_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pmc_b16/gemm_ab.log; exit $rc
