#!/bin/bash
# Full-size training-trajectory parity: fused HIP path vs PyTorch fp32 reference (scripts/convergence_check.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/conv
timeout -k 10 300 python -u scripts/convergence_check.py --steps 400 --lr 1e-4 > gpurun_out/conv/b16_lr1e-4.log 2>&1 || exit $?
tail -1 gpurun_out/conv/b16_lr1e-4.log
timeout -k 10 300 python -u scripts/convergence_check.py --steps 200 --lr 1e-3 > gpurun_out/conv/b16_lr1e-3.log 2>&1 || exit $?
tail -1 gpurun_out/conv/b16_lr1e-3.log
