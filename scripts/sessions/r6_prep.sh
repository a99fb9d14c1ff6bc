#!/bin/bash
# Round 6: attention backward pre-pass with XCD-contiguous (batch, head) pairs vs round-robin:
# kernel checks, isolated backward A/B at the ViT-H/14 and ViT-L/16@384 shapes, H/14 fp8 bench pair.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-prep}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 300 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run 300 attn_ab.log python scripts/attn_ab.py --shapes h14,l16_384 --ab prepxcd --bwd --rounds 5
grep "attn bwd" "$O/attn_ab.log"
