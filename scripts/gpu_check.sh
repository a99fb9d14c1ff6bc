#!/bin/bash
# Standard check session: every GPU test (pytest -m gpu), smoke, the headline bench (twice) and an
# in-step / serialized rocprofv3 kernel profile of the bench (scripts/gpu_prof_step.sh <tag>).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-chk}"
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-6} "$R/gpurun_out/$log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 600 ${TAG}_pytest.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
TAILN=1 run 180 ${TAG}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 run 200 ${TAG}_bench1.log python bench.py --steps 20 --warmup 5
TAILN=1 run 200 ${TAG}_bench2.log python bench.py --steps 20 --warmup 5
[ "${PROF:-1}" = 1 ] && bash scripts/gpu_prof_step.sh $TAG
exit 0
