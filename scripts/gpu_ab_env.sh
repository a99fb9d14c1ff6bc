#!/bin/bash
# A/B over several values of one env var, alternating, same box.
# usage: gpurun -- bash scripts/gpu_ab_env.sh VAR "v1 v2 ..." [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/abenv
VAR="$1"; VALS="$2"; shift 2
for i in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/abenv/run.log 2>&1 || exit $?
    echo "$VAR=$v $(tail -1 gpurun_out/abenv/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
