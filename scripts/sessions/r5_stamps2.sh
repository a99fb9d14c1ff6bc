#!/bin/bash
# Round 5: GEMM epilogue stamps with the register-direct epilogue split (row 0 | rows 1-7 | tail)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5e; mkdir -p $O; export TMPDIR=/tmp
for e in bias resid gelu dgelu; do
  timeout -k 10 120 python -u scripts/gemm_stamps.py --epi $e --tiles 256,2304 > $O/stamps_$e.log 2>&1 || { tail -5 $O/stamps_$e.log; exit 1; }
  cat $O/stamps_$e.log
done
