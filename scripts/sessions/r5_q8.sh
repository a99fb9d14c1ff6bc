#!/bin/bash
# Round 5: the attention backward writes dQKV's e5m2 copy with bf16 weight gradients too (no quantize
# pass before the fp8 qkv dgrad): kernel checks, ViT-H/14 fp8 alternating against the previous recipe
# (ab_prev/), and its steady-state step table.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5q8}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 600 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do
  step 300 h14_new_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
  PVR_PKG_ROOT=$R/ab_prev step 300 h14_prev_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/h14_prof" -o step --output-format csv -- python3 "$R/bench.py" --model vit_h14 --dtype fp8 --steps 3 --warmup 2 --serial-wgrad > "$R/$O/h14_prof.log" 2>&1; rc=$?
cd "$R"; echo "[h14 prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/steady_step.py "$(find "$O/h14_prof" -name "*kernel_trace.csv" | head -n1)" "ViT-H/14 b256 fp8 (bf16 wgrad)" > "$O/h14_steady.md"
rm -rf "$O/h14_prof"
head -n 3 "$O/h14_steady.md" | tail -n 1
