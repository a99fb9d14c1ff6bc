#!/bin/bash
# Round 5 checkpoint: GPU suite (resume / odd patch / pruned knobs), GEMM epilogue stamps, bench
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for e in bias resid gelu dgelu; do
  timeout -k 10 120 python -u scripts/gemm_stamps.py --epi $e > $O/stamps_$e.log 2>&1 || { tail -5 $O/stamps_$e.log; exit 1; }
  cat $O/stamps_$e.log
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
tail -n1 $O/bench.log | cut -c1-220
