#!/bin/bash
# Verification session: pytest -m gpu, smoke, headline bench, rocprofv3 kernel stats of the bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-4} "$R/gpurun_out/$log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 700 pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 180 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench.log python bench.py --steps 20 --warmup 5
[ "${PROF:-1}" = 1 ] && run 300 prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 3
exit 0
