#!/bin/bash
# fp8 dgrad GEMMs (enable_fp8(dgrad=True)): GPU tests (incl. check_vit_fp8_dgrad), then ViT-H/14 fp8 bench A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/f8d; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/f8d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/f8d/pytest.log; grep -h "fp8 dgrad" gpurun_out/f8d/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --model vit_h14 --batch 128 --dtype fp8 $([ "$v" = 0 ] && echo --fp8-bf16-dgrad) --steps 8 --warmup 3 > gpurun_out/f8d/h14_${v}_$i.log 2>&1
    rc=$?; echo "h14 fp8 dgrad=$v #$i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/f8d/h14_${v}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/f8d/h14_${v}_$i.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
