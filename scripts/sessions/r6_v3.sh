#!/bin/bash
# Round 6, late: GPU suite with e4m3 as the fp8 gradient default, LayerNorm fp8-forward grid A/B,
# ViT-H/14 fp8 default bench and kernel table.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-v3}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run 120 ln_ab.log python scripts/ln_ab.py --caps 4,8,16 --rounds 4
cat "$O/ln_ab.log"
run 400 h14_fp8.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d "$R/$O/h14_prof" -o step --output-format csv -- python3 "$R/bench.py" --model vit_h14 --dtype fp8 --steps 3 --warmup 3 --serial-wgrad > "$R/$O/h14_prof.log" 2>&1 || exit $?
cd "$R"; python scripts/steady_step.py "$(find "$O/h14_prof" -name "*kernel_trace.csv" | head -n1)" "ViT-H/14 b256 fp8 (e4m3 gradients, fp8 wgrad)" > "$O/h14_steady.md"
rm -rf "$O/h14_prof"; grep -v "^$" "$O/h14_steady.md" | head -20
