#!/bin/bash
# ViT-H/14 224: fused bf16 vs fused fp8 (enable_fp8) trajectories, same init and batches (no PyTorch paths: too slow).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/conv
timeout -k 10 500 python -u scripts/convergence_check.py --model vit_h14 --steps 600 --batch 32 --lr 1e-4 --fp8 --no-reference --log 20 > gpurun_out/conv/h14_fp8_vs_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/conv/h14_fp8_vs_bf16.log
