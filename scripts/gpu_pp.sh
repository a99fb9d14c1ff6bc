#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-12} "$R/gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 600 pytest_gpu.log python -m pytest tests -m gpu -x -q -p no:cacheprovider
run 300 bench.log python bench.py --steps 20 --warmup 5
TAILN=30 run 200 stamps.log python scripts/gemm_stamps.py
