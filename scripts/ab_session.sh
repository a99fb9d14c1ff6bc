#!/bin/bash
# A/B session: tail split numerics, bench A/Bs, GEMM table vs hipBLASLt, GPU test suite.
# Every GPU step under its own timeout; the first failure ends it.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step 300 tail_check.log python -u scripts/tail_check.py
step 200 bench_on1.log python bench.py
step 200 bench_off1.log python bench.py --no-gemm-tail
step 200 bench_on2.log python bench.py
step 200 bench_off2.log python bench.py --no-gemm-tail
step 200 bench_win0.log python bench.py --side-window 0
step 400 gemm_ab_tail.log python -u scripts/gemm_ab.py --ab tail --rounds 3
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
