#!/bin/bash
# Numerics of every kernel, then A/B of the attention / wgrad changes: kernel microbench
# (whole-head vs tiled forward), full-step benches (default, tiled forward, high-priority main stream).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-3} "$R/gpurun_out/$log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=12 run 400 checks.log python tests/kernel_checks.py
TAILN=14 run 300 kb_new.log python scripts/bench_kernels.py --tiles 12 --only gemm,attn
TAILN=4 PVR_ATTN_FWD_TILED=1 run 200 kb_tiled.log python scripts/bench_kernels.py --tiles 12 --only attn
run 300 bench.log python bench.py --steps 20 --warmup 5
PVR_ATTN_FWD_TILED=1 run 300 bench_tiled.log python bench.py --steps 20 --warmup 5
run 300 bench_prio.log python bench.py --steps 20 --warmup 5 --main-prio -1
exit 0
