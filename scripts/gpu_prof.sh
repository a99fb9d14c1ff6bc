#!/bin/bash
# GPU session 2: kernel microbenchmarks, reference-style eager baseline, rocprofv3 kernel stats.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-60} "$R/gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
run 500 kbench.log python scripts/bench_kernels.py
run 300 bench_torch.log python bench.py --impl torch --steps 10 --warmup 3
export TMPDIR=/tmp
cd /tmp
TAILN=5 run 400 rocprof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2
cd "$R"
ls -R gpurun_out/prof | head -20
