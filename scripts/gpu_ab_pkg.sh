#!/bin/bash
# A/B of two builds on one box: the tree's package vs an alternative build (default ab_old/), alternating.
# usage: gpurun -- bash scripts/gpu_ab_pkg.sh [alt root] [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/abpkg
ALT="${1:-ab_old}"; shift
for i in 1 2; do
  for v in . "$ALT"; do
    timeout -k 10 300 python scripts/bench_pkg.py "$v" --steps 20 --warmup 5 "$@" > gpurun_out/abpkg/run.log 2>&1 || exit $?
    echo "pkg=$v $(grep bench_pkg gpurun_out/abpkg/run.log | cut -c1-80) $(tail -1 gpurun_out/abpkg/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
