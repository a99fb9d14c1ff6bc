#!/bin/bash
# Persistent ping-pong (tile 13) with the register-direct epilogue and counted tile-boundary waits
# vs one tile per workgroup (12): GEMM numerics, per-epilogue kernel timing, bench A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-14} "$R/gpurun_out/$log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 200 pd_checks.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 pd_kb.log python -u scripts/bench_kernels.py --only epi --epi-tiles 12,13 --gelu-tiles "" --rounds 2
for i in 1 2; do
  PVR_PERSISTENT=0 PVR_GELU_TILE=12 run 200 pd_bench_t12_$i.log python bench.py --steps 20 --warmup 5
  PVR_PERSISTENT=1 run 200 pd_bench_t13_$i.log python bench.py --steps 20 --warmup 5
  PVR_PERSISTENT=0 run 200 pd_bench_gelu13_$i.log python bench.py --steps 20 --warmup 5
done
exit 0
