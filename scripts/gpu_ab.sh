#!/bin/bash
# A/B: bench with env VAR=A vs VAR=B, alternating, same box.  usage: AB_VAR=PVR_X AB_A=1 AB_B=0 bash scripts/gpu_ab.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
for i in 1 2; do
  for v in "$AB_A" "$AB_B"; do
    env "$AB_VAR=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || exit $?
    echo "$AB_VAR=$v $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
