R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/f8e; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/f8e/pytest.log 2>&1 && tail -1 gpurun_out/f8e/pytest.log && \
timeout -k 10 200 python bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 8 --warmup 3 > gpurun_out/f8e/h14.log 2>&1 && tail -1 gpurun_out/f8e/h14.log | cut -c1-400 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/f8e/b16.log 2>&1 && tail -1 gpurun_out/f8e/b16.log | cut -c1-200
