#!/bin/bash
# A/B session (round 4): attention forward numerics + A/B, bench variants on one box, H/14 memory,
# GPU test suite. Every GPU step under its own timeout; the first failure ends it.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
step 300 attn_fwd_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "numerics" -x
step 300 attn_ab.log python -u scripts/attn_ab.py --ab fwd_qg --bwd
for r in 1 2; do
  step 200 b_def_$r.log python bench.py
  step 200 b_notail_$r.log python bench.py --no-gemm-tail
  step 200 b_hold0_$r.log python bench.py --side-hold-gb 0
done
step 300 h14_def.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
step 300 h14_hold0.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4 --side-hold-gb 0
step 300 l16_def.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 6 --warmup 3
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/h14_prof" -o step --output-format csv -- python3 "$R/bench.py" --model vit_h14 --dtype fp8 --batch 256 --steps 4 --warmup 3 --serial-wgrad > "$R/$O/h14_prof.log" 2>&1; rc=$?
cd "$R"; echo "[h14 prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
S=$(find "$O/h14_prof" -name "*kernel_stats.csv" | head -n1); python scripts/summarize_prof.py "$S" 7 "ViT-H/14 fp8 b256 kernel stats (r4, serial)" > "$O/h14_kernel_stats_serial.md" 2>&1
