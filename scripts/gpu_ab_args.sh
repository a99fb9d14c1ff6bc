#!/bin/bash
# A/B of bench argument sets, alternating, same box: gpu_ab_args.sh "<args A>" "<args B>" [more...]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/abargs
for i in 1 2; do
  for a in "$@"; do
    timeout -k 10 400 python bench.py --steps 10 --warmup 3 $a > gpurun_out/abargs/run.log 2>&1 || exit $?
    echo "[$a] $(tail -1 gpurun_out/abargs/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
