#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ab7
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x > gpurun_out/ab7/attn_checks.log 2>&1; rc=$?; echo "[checks] rc=$rc"; tail -1 gpurun_out/ab7/attn_checks.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/attn_ab.py --ab fwd_qg --bwd > gpurun_out/ab7/attn_ab.log 2>&1; rc=$?; echo "[attn_ab] rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash scripts/pmc_attn.sh ab7/pmc_h14 h14 && timeout -k 10 300 bash scripts/pmc_attn.sh ab7/pmc_l16 l16_384 && timeout -k 10 300 bash scripts/pmc_attn.sh ab7/pmc_b16 b16
for lr in 3e-5 1e-5; do
  timeout -k 10 240 python -u scripts/convergence_check.py --model vit_h14 --steps 300 --batch 64 --lr $lr --no-reference --log 50 > gpurun_out/ab7/conv_h14_lr$lr.log 2>&1; rc=$?; echo "[conv lr $lr] rc=$rc"; tail -1 gpurun_out/ab7/conv_h14_lr$lr.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/fp8_vs_scaled_mm.py > gpurun_out/ab7/fp8_vs_scaled_mm.log 2>&1; rc=$?; echo "[scaled_mm] rc=$rc"; [ $rc -eq 0 ] || exit $rc
