#!/bin/bash
# Round 5: attention backward pre-pass with the lse load hoisted into the row-load batch: kernel
# checks, backward times at the BASELINE shapes, and a kernel trace of the ViT-L/16-384 / ViT-H/14
# backward (body / tail / pre-pass launches separately).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5prep}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep "bwd\|passed\|failed" "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step 200 attn_ab.log python scripts/attn_ab.py --bwd --rounds 3 --shapes l16_384,h14
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/attn_prof" -o attn --output-format csv -- python3 "$R/scripts/attn_ab.py" --bwd --rounds 1 --shapes l16_384,h14 > "$R/$O/attn_prof.log" 2>&1; rc=$?
cd "$R"; echo "[attn prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
