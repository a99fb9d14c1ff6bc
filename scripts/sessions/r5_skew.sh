#!/bin/bash
# Round 5: first-round workgroup start skew (desynchronise the CUs' epilogue store / load bursts)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/gemm_ab.py --ab skew:0,4000,8000,16000 --rounds 4 --only fwd,dgrad > $O/gemm_skew.log 2>&1
rc=$?; cat $O/gemm_skew.log; exit $rc
