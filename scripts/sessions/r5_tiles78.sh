#!/bin/bash
# Round 5: two-workgroups-per-CU GEMM tiles (7 = 128x256, 8 = 256x128, 4 waves, BK 32, 3-stage ring)
# vs the default selection: numerics checks, then every ViT-B/16 b256 GEMM interleaved.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/run_checks.py check_gemm_fwd,check_gemm_gelu,check_gemm_dgelu,check_gemm_dgrad > $O/checks.log 2>&1
rc=$?; tail -n 40 $O/checks.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/gemm_ab.py --ab tiles:def,7,8 --rounds 4 --only fwd,dgrad > $O/gemm_ab.log 2>&1
rc=$?; cat $O/gemm_ab.log; exit $rc
