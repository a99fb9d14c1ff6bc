#!/bin/bash
# Round 6: learning-phase seed study of e4m3 vs e5m2 gradients (fp8 forward + dgrad + wgrad) against
# bf16, the same protocol as profiles/r6/fp8_study (ViT-H/14, batch 64, lr 1e-5, 1000-step schedule
# trained to step 600, 20-step windows ending at 200 / 400 / 600). Usage: r6_e4m3_study.sh OUT SEED_START
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-e4m3_study}; mkdir -p "$O"; S=${2:-0}
timeout -k 10 1100 python -u scripts/convergence_check.py --model vit_h14 --steps 1000 --stop-at 600 --lr 1e-5 --batch 64 \
  --fp8-study 3 --seed-start "$S" --checkpoints 200,400,600 --window 20 --variants fused,fused_fp8w,fused_fp8w4 \
  > "$O/seeds$S.log" 2>&1; rc=$?
grep "\[study\]" "$O/seeds$S.log"; exit $rc
