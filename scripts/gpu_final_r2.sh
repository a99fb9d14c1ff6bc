#!/bin/bash
# End-of-session check: every GPU test, smoke, headline bench, then the fp8 trajectory comparison.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O="$R/gpurun_out/fin2"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
tail -1 "$O/smoke.log"
timeout -k 10 240 python bench.py > "$O/bench.log" 2>&1 || exit $?
tail -1 "$O/bench.log" | cut -c1-200
bash scripts/gpu_convergence_fp8.sh
