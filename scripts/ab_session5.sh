#!/bin/bash
# GPU session: kernel checks, BASELINE benches, one H/14 fp8 steady-step kernel table (round 4)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 600 kernel_checks.log python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
step 300 h14_def.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
step 200 b_def.log python bench.py
step 300 l16_def.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 6 --warmup 3
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/h14_prof" -o step --output-format csv -- python3 "$R/bench.py" --model vit_h14 --dtype fp8 --batch 256 --steps 3 --warmup 2 --serial-wgrad > "$R/$O/h14_prof.log" 2>&1; rc=$?
cd "$R"; echo "[h14 prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/steady_step.py "$(find "$O/h14_prof" -name "*kernel_trace.csv" | head -n1)" "ViT-H/14 fp8 b256" > "$O/h14_steady.md"
rm -rf "$O/h14_prof"
head -n 14 "$O/h14_steady.md"
