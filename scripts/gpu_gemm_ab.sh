#!/bin/bash
# GEMM change check: kernel numerics (pytest -m gpu kernel checks), per-epilogue timing on tiles 12/13,
# and the headline bench (twice).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-14} "$R/gpurun_out/$log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 200 ga_checks.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 ga_kb.log python -u scripts/bench_kernels.py --only epi --epi-tiles 12,13 --gelu-tiles "" --rounds 2
TAILN=1 run 200 ga_bench1.log python bench.py --steps 20 --warmup 5
TAILN=1 run 200 ga_bench2.log python bench.py --steps 20 --warmup 5
exit 0
