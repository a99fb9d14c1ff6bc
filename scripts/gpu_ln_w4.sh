#!/bin/bash
# LayerNorm backward on 4-column chunks (D = 768 / 1280): checks, kernel timing per variant, step A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/lnw4; mkdir -p $O; export TMPDIR=/tmp
for v in 1 2 0; do
  PVR_LN_BWD_W4=$v timeout -k 10 120 python scripts/run_checks.py check_layernorm,check_vit_block_link > $O/checks_$v.log 2>&1; rc=$?
  echo "== W4=$v checks"; cat $O/checks_$v.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
  PVR_LN_BWD_W4=$v timeout -k 10 120 python scripts/bench_kernels.py --only ln > $O/kb_$v.log 2>&1 || exit $?
  grep ln_ $O/kb_$v.log
done
for i in 1 2; do
  for v in 0 1 2; do
    PVR_LN_BWD_W4=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/ab.log 2>&1 || exit $?
    echo "PVR_LN_BWD_W4=$v $(tail -1 $O/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
