#!/bin/bash
# Round 5: the round-end checks as the driver runs them (GPU suite, smoke) plus the headline bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5full}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 1100 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 200 bench.log python bench.py
