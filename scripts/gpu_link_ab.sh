#!/bin/bash
# Numerics (incl. the linked LayerNorm-backward dropout path), then A/B of the block link.
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
TAILN=6 run 400 checks.log python tests/kernel_checks.py
run 300 bench.log python bench.py --steps 20 --warmup 5
PVR_BLOCK_LINK=0 run 300 bench_nolink.log python bench.py --steps 20 --warmup 5
run 300 bench2.log python bench.py --steps 20 --warmup 5
exit 0
