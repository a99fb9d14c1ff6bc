#!/bin/bash
# Trajectory check of the fp8 GEMM path (enable_fp8) next to bf16 fused / fp32 / autocast-bf16 (ViT-B/16 224).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/conv
timeout -k 10 400 python -u scripts/convergence_check.py --steps 400 --lr 1e-4 --fp8 > gpurun_out/conv/b16_lr1e-4_fp8.log 2>&1 || exit $?
tail -1 gpurun_out/conv/b16_lr1e-4_fp8.log
