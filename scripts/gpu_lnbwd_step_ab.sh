#!/bin/bash
# In-step A/B of the LayerNorm-backward grid cap (the isolated kbench picked 512; in the step the
# kernel shares the GPU with the side-stream weight-gradient GEMMs).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/lnab; export TMPDIR=/tmp
for i in 1 2; do
  for nb in 512 1024 768 384; do
    PVR_LN_BWD_BLOCKS=$nb timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/lnab/b_${nb}_$i.log 2>&1
    rc=$?; echo "ln_bwd_blocks=$nb #$i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/lnab/b_${nb}_$i.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
