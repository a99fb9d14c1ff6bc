#!/bin/bash
# One GPU session: kernel numerics -> smoke -> short bench. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpu_out_tmp gpurun_out
run() {  # run <seconds> <logfile> <cmd...>; numerics failures (exit 1) do not stop the session
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n 40 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 420 checks.log python tests/kernel_checks.py
run 180 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench.log python bench.py --steps 10 --warmup 3
