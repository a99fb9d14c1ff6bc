#!/bin/bash
# kernel checks (incl. dh=80 attention, ViT-H-like fused model) -> bench B/16 -> short L/16@384 and H/14 runs
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-40} "$R/gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 420 checks.log python tests/kernel_checks.py
run 300 bench.log python bench.py --steps 20 --warmup 5
run 300 bench_l16_384.log python bench.py --model vit_l16 --image-size 384 --batch 32 --steps 5 --warmup 2
run 300 bench_h14.log python bench.py --model vit_h14 --batch 64 --steps 5 --warmup 2
