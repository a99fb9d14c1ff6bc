#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-3} "$R/gpurun_out/$log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=8 run 300 kbench_fp8.log python scripts/bench_kernels.py --only fp8
run 300 bench_h14.log python bench.py --model vit_h14 --batch 128 --steps 5 --warmup 2
run 300 bench_h14_fp8.log python bench.py --model vit_h14 --batch 128 --steps 5 --warmup 2 --dtype fp8
run 300 bench_b16_fp8.log python bench.py --steps 10 --warmup 3 --dtype fp8
