#!/bin/bash
# Small-M split-K forward GEMMs (serving): checks, latency A/B at batch 1 / 8 / 32 / 256.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/sks; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 180 python scripts/run_checks.py check_gemm_small_splitk,check_vit_inference,check_vit_fused_vs_reference > $O/checks.log 2>&1; rc=$?
grep -v amdgpu.ids $O/checks.log; [ $rc -eq 0 ] || exit $rc
for b in 1 8 32 256; do
  for v in 0 1; do
    PVR_SMALL_SPLITK=$v timeout -k 10 300 python bench.py --infer --batch $b --steps 50 --warmup 10 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "infer b$b PVR_SMALL_SPLITK=$v: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms")')"
  done
done
