#!/bin/bash
# GPU session: full GPU suite + smoke on the final tree
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-final3}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 200 b_def.log python bench.py
