#!/bin/bash
# Round 5: epilogue-input prefetch (dGELU factor / residual LDS-DMA'd to a junk slot mid K loop)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/run_checks.py check_gemm_fwd,check_gemm_dgelu,check_gemm_tail_split,check_gemm_dropout > $O/checks.log 2>&1
rc=$?; tail -n 12 $O/checks.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/gemm_ab.py --ab pf --rounds 6 --only fwd,dgrad > $O/gemm_pf.log 2>&1
rc=$?; cat $O/gemm_pf.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_pf_on_$i.log 2>&1 || exit $?
PVR_GEMM_PREFETCH=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_pf_off_$i.log 2>&1 || exit $?
done
tail -n1 $O/bench_pf_*.log | cut -c1-200
