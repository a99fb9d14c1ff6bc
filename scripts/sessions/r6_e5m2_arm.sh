#!/bin/bash
# Round 6: the e5m2-gradient arm (fp8 forward + dgrad + wgrad) for seeds 6-11 of the e4m3 study (whose
# own "fused_fp8w" arm ran e4m3 after the default switch); same protocol as r6_e4m3_study.sh.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-e4m3_study}; mkdir -p "$O"
timeout -k 10 1100 python -u scripts/convergence_check.py --model vit_h14 --steps 1000 --stop-at 600 --lr 1e-5 --batch 64 \
  --fp8-study 6 --seed-start 6 --checkpoints 200,400,600 --window 20 --variants fused_fp8w \
  > "$O/seeds6-11_e5m2.log" 2>&1; rc=$?
grep "\[study\]" "$O/seeds6-11_e5m2.log"; exit $rc
