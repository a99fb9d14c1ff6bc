#!/bin/bash
# Head kernels: numerics checks + one in-step profile of the bench (head kernel times).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/hd_checks.log 2>&1 || { tail -30 gpurun_out/hd_checks.log; exit 1; }
tail -2 gpurun_out/hd_checks.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/hd_bench.log 2>&1 || exit 1
tail -1 gpurun_out/hd_bench.log | cut -c1-200
PROF=1 bash scripts/gpu_prof_step.sh hd 2>&1 | grep -E "head|xent|scale_by|metrics|mean_k|Cijk|native|rocclr|step " | cut -c1-160
