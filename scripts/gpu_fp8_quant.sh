#!/bin/bash
# fp8 activation-quantizer change: kernel numerics (all kernel checks, fp8 ones included), the
# quantizer microbench, then the fp8 and bf16 B/16 benches on the same box.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-3} "$R/gpurun_out/$log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=2 run 300 checks.log python -u tests/kernel_checks.py
TAILN=8 run 300 kbench_fp8.log python scripts/bench_kernels.py --only fp8
run 300 bench_b16_fp8.log python bench.py --steps 10 --warmup 3 --dtype fp8
run 300 bench.log python bench.py --steps 20 --warmup 5
exit 0
