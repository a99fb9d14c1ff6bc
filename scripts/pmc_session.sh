#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ab7
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x > gpurun_out/ab7/attn_checks.log 2>&1; rc=$?; echo "[checks] rc=$rc"; tail -1 gpurun_out/ab7/attn_checks.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/attn_ab.py --ab fwd_qg --bwd > gpurun_out/ab7/attn_ab.log 2>&1; rc=$?; echo "[attn_ab] rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash scripts/pmc_attn.sh ab7/pmc_h14 h14 && timeout -k 10 300 bash scripts/pmc_attn.sh ab7/pmc_l16 l16_384 && timeout -k 10 300 bash scripts/pmc_attn.sh ab7/pmc_b16 b16
