#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-80} "$R/gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP"; exit $rc; fi; }
run 400 checks2.log python tests/kernel_checks.py
#run 400 kbench2.log python scripts/bench_kernels.py --tiles 0,6 --only gemm
run 300 bench.log python bench.py --steps 10 --warmup 3
