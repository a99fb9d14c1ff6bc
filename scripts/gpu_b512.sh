#!/bin/bash
# Kernel checks, the headline bench, and the per-GPU config of the multi-GPU runs (b512) with and
# without the DDP wrapper (world 1), to separate batch-size effects from gradient-transport cost.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-2} "$R/gpurun_out/$log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 300 checks.log python -u tests/kernel_checks.py
run 300 bench.log python bench.py --steps 20 --warmup 5
run 300 bench_b512.log python bench.py --steps 10 --warmup 3 --batch 512
run 300 bench_b512_ddp.log python bench.py --steps 10 --warmup 3 --batch 512 --force-ddp
exit 0
