#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/fin; export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 && tail -1 gpurun_out/fin/smoke.log && \
timeout -k 10 200 python bench.py > gpurun_out/fin/bench_default.log 2>&1 && tail -1 gpurun_out/fin/bench_default.log | cut -c1-250 && \
timeout -k 10 200 python bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 8 --warmup 3 > gpurun_out/fin/h14_fp8.log 2>&1 && tail -1 gpurun_out/fin/h14_fp8.log | cut -c1-400
