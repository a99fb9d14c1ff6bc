#!/bin/bash
# Round 5: attention backward pre-pass with 8 lanes per query row (in-tree) vs 16 (ab_head/): kernel
# checks, backward times alternating, kernel traces of both (pre-pass launch time), ViT-H/14 fp8 step.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5prep8}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "bwd\|passed\|failed\|images/sec" "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 200 attn_base_$i.log python scripts/attn_ab.py --bwd --rounds 3
  step 200 attn_new_$i.log python scripts/attn_ab.py --bwd --rounds 3
done
for v in new base; do
  cd /tmp
  if [ $v = base ]; then export PVR_PKG_ROOT=$R/ab_head; else unset PVR_PKG_ROOT; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$v" -o attn --output-format csv -- python3 "$R/scripts/attn_ab.py" --bwd --rounds 1 > "$R/$O/prof_$v.log" 2>&1; rc=$?
  cd "$R"; echo "[prof $v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
unset PVR_PKG_ROOT
for i in 1 2; do
  PVR_PKG_ROOT=$R/ab_head step 300 h14_base_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
  step 300 h14_new_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 10 --warmup 3
done
