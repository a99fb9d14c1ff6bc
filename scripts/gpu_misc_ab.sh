#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof5
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-2} "$R/gpurun_out/$log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=3 run 400 checks.log python tests/kernel_checks.py
run 300 bench.log python bench.py --steps 20 --warmup 5
export TMPDIR=/tmp
cd /tmp
TAILN=1 run 300 prof5/run.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof5" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 3
exit 0
