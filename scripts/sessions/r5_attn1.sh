#!/bin/bash
# Round 5: attention backward (pipelined B/16 kernel) with the block stores left in flight
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/run_checks.py check_attn_bwd,check_vit > $O/checks.log 2>&1
rc=$?; tail -n 30 $O/checks.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/attn_ab.py --shapes b16,l16_384,h14 --bwd --rounds 4 > $O/attn.log 2>&1 || exit $?
cat $O/attn.log
timeout -k 10 400 python -u scripts/gemm_ab.py --rounds 3 --only "dGELU,fc1 fwd,colsum" > $O/gemm_epi.log 2>&1 || exit $?
cat $O/gemm_epi.log
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || exit $?; tail -n1 $O/bench$i.log | cut -c1-200; done
