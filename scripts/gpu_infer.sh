#!/bin/bash
# Inference path: checks, serving throughput (eval forward, inference_mode) at ViT-B/16 b256 / b1024, L/16-384.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/infer; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 180 python scripts/run_checks.py check_vit_inference,check_vit_fused_vs_reference,check_gemm_gelu > $O/checks.log 2>&1; rc=$?
grep -v amdgpu.ids $O/checks.log; [ $rc -eq 0 ] || exit $rc
for args in "--batch 256" "--batch 1024" "--model vit_l16 --image-size 384 --batch 128" "--model vit_h14 --batch 256"; do
  timeout -k 10 300 python bench.py --infer --steps 20 --warmup 5 $args > $O/b.log 2>&1 || exit $?
  echo "infer $args: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
