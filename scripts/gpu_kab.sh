#!/bin/bash
# GPU kernel checks, then an alternating attention microbenchmark A/B of this tree vs an alternative
# package copy (default ab_old/, holding its own scripts/), at the given N,H,dh:batch shapes.
# usage: gpurun -- bash scripts/gpu_kab.sh [alt root] 577,16,64:64 257,16,80:64 ...
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/kab; export TMPDIR=/tmp
ALT="${1:-ab_old}"; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kab/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/kab/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for shp in "$@"; do
    for v in . "$ALT"; do
      timeout -k 10 120 python "$v/scripts/bench_kernels.py" --only attn --attn-shape "${shp%%:*}" --batch "${shp##*:}" > gpurun_out/kab/kb.log 2>&1 || exit $?
      echo "$v $shp $(grep attn_ gpurun_out/kab/kb.log | tr -s ' ' | tr '\n' '|')"
    done
  done
done
exit 0
