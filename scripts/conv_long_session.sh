#!/bin/bash
# GPU session: longer ViT-H/14 learning-phase study (fp8 vs bf16, 3 seeds, 1000 steps at lr 1e-5)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/conv_long; export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/convergence_check.py --model vit_h14 --fp8-study 3 --steps 1000 --batch 64 --lr 1e-5 --log 100 > gpurun_out/conv_long/h14_fp8_study_1000.log 2>&1
rc=$?; tail -n 5 gpurun_out/conv_long/h14_fp8_study_1000.log; exit $rc
