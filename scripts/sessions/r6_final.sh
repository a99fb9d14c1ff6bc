#!/bin/bash
# Round 6, last tree: GPU suite, smoke, headline bench x2, H/14 fp8 (e4m3 default), fp8 serving.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-final}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2; do run 240 b16_$i.log python bench.py; done
run 500 h14_fp8_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --force-ddp --steps 8 --warmup 4
run 300 h14_fp8_infer.log python bench.py --infer --model vit_h14 --dtype fp8 --steps 10 --warmup 3
