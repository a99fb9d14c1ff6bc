#!/bin/bash
# GPU test tier + the 4-column LayerNorm backward at D = 1280 (ViT-H/14 fp8 step A/B).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/lnw4h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    PVR_LN_BWD_W4=$v timeout -k 10 300 python bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 8 --warmup 3 > $O/ab.log 2>&1 || exit $?
    echo "H14 fp8 PVR_LN_BWD_W4=$v $(tail -1 $O/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
