#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-2} "$R/gpurun_out/$log" | cut -c1-330
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=15 run 300 pytest_train.log python -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider
run 300 bench_graph.log python bench.py --steps 20 --warmup 5 --graph
run 300 bench_b32.log python bench.py --steps 30 --warmup 5 --batch 32
run 300 bench_b32_graph.log python bench.py --steps 30 --warmup 5 --batch 32 --graph
