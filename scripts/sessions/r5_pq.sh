#!/bin/bash
# Round 5: persistent whole-head attention backward grid (ViT-B/16): one workgroup per CU (in-tree)
# vs 0.75x / 0.5x the CUs (ab_pq3/, ab_pq2/: -DPVR_PIPE8_GRID_Q=3/2), so the pairs rebalance when
# side-stream weight gradients hold some CUs.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5pq}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|bwd b16 .*TF' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; }
PVR_PKG_ROOT=$R/ab_pq2 step 400 kernels_pq2.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 200 attn_base_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes b16
  for v in pq3 pq2; do PVR_PKG_ROOT=$R/ab_$v step 200 attn_${v}_$i.log python scripts/attn_ab.py --bwd --rounds 3 --shapes b16; done
done
for i in 1 2 3; do
  step 200 b16_base_$i.log python bench.py
  for v in pq3 pq2; do PVR_PKG_ROOT=$R/ab_$v step 200 b16_${v}_$i.log python bench.py; done
done
