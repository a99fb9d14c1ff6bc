#!/bin/bash
# Register-direct vs LDS-staged ping-pong GEMM epilogue: GEMM numerics checks, per-epilogue kernel
# timing and the headline bench, A/B on one box (PVR_EPI_STAGED=1 / 0).
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
run 200 ed_checks.log python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "not nothing"
for i in 1 2; do
  PVR_EPI_STAGED=1 run 200 ed_kb_staged$i.log python -u scripts/bench_kernels.py --only epi --epi-tiles 12 --gelu-tiles ""
  PVR_EPI_STAGED=0 run 200 ed_kb_direct$i.log python -u scripts/bench_kernels.py --only epi --epi-tiles 12 --gelu-tiles ""
done
for i in 1 2; do
  PVR_EPI_STAGED=1 run 200 ed_bench_staged$i.log python bench.py --steps 20 --warmup 5
  PVR_EPI_STAGED=0 run 200 ed_bench_direct$i.log python bench.py --steps 20 --warmup 5
done
exit 0
