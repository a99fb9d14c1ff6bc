#!/bin/bash
# Round 5, last check of the final tree: GPU suite, smoke, headline bench, and rocprofv3 --stats of
# the default (side-stream) ViT-B/16 b256 run.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5last}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; }
step 1100 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 200 bench_1.log python bench.py
step 200 bench_2.log python bench.py
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o b16 --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/$O/prof.log" 2>&1; rc=$?
cd "$R"; echo "[prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -n1); cp "$f" "$O/b16_side_kernel_stats.csv"; rm -rf "$O/prof"
