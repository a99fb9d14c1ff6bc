#!/bin/bash
# Round 5: tail-split attention backward with the body slabs added in the tail's dQ epilogue (mode 5)
# vs HEAD (ab_prev/): kernel checks, backward times alternating, ViT-L/16-384 step alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5tail5}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "bwd l16\|bwd h14\|passed\|failed\|\"value\"" "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 200 ab_new_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
  PVR_PKG_ROOT=$R/ab_prev step 200 ab_prev_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
done
for i in 1 2; do
  step 300 l16_new_$i.log python bench.py --model vit_l16 --image-size 384 --steps 6 --warmup 3
  PVR_PKG_ROOT=$R/ab_prev step 300 l16_prev_$i.log python bench.py --model vit_l16 --image-size 384 --steps 6 --warmup 3
done
