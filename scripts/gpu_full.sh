#!/bin/bash
# Full GPU session: pytest -m gpu -> smoke -> bench (fused + eager torch) -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout ends the session.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof
run() {  # run <seconds> <logfile> <cmd...>; test failures (rc 1) do not stop the session
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-30} "$R/gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 600 pytest_gpu.log python -m pytest tests -m gpu -x -q -p no:cacheprovider
run 180 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench.log python bench.py --steps 20 --warmup 5
[ -n "$SKIP_TORCH" ] || run 300 bench_torch.log python bench.py --impl torch --steps 10 --warmup 3
export TMPDIR=/tmp
cd /tmp
TAILN=5 run 400 rocprof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2
