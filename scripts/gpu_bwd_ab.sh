#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-2} "$R/gpurun_out/$log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=3 run 400 checks.log python tests/kernel_checks.py
TAILN=2 run 200 kb_attn_new.log python scripts/bench_kernels.py --only attn
TAILN=2 PVR_ATTN_BWD_FUSED=1 run 200 kb_attn_old.log python scripts/bench_kernels.py --only attn
run 300 bench.log python bench.py --steps 20 --warmup 5
PVR_ATTN_BWD_FUSED=1 run 300 bench_oldbwd.log python bench.py --steps 20 --warmup 5
exit 0
