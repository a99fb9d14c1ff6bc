#!/bin/bash
# Round 6: e4m3 gradients in the fp8 backward (enable_fp8(grad_fmt="e4m3")): kernel checks (the whole
# kernel-check list, the fmt=0 rows included), smoke, ViT-H/14 fp8 b256 with e5m2 vs e4m3 gradients
# alternating (same kernels, so equal speed is expected), headline bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-e4m3}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 900 kernels.log python -u -m pytest tests/test_gpu_kernels.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider
grep "fp8 gradient formats\|e4m3" "$O/kernels.log" | cut -c1-220 | head -20
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2; do
  run 400 h14_e5m2_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
  run 400 h14_e4m3_$i.log python bench.py --model vit_h14 --dtype fp8 --fp8-grad e4m3 --steps 8 --warmup 4
done
run 240 b16.log python bench.py
