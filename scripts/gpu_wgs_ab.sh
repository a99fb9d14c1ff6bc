#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for w in 256 192 128 256 160; do
  PVR_WGRAD_WGS=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_wgs$w.log 2>&1 || exit $?
  echo "wgs $w: $(grep -o '"value": [0-9.]*' gpurun_out/bench_wgs$w.log)"
done
