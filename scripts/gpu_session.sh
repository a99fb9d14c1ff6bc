#!/bin/bash
# One GPU session: GPU tests, smoke, headline bench, rocprofv3 kernel stats of the headline step.
# Usage (from the container): gpurun --timeout 900 -- bash scripts/gpu_session.sh <tag> [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
TAG="${1:-s}"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
tail -1 "$O/smoke.log"
timeout -k 10 240 python bench.py "$@" > "$O/bench.log" 2>&1 || exit $?
tail -1 "$O/bench.log" | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 3 "$@" > "$O/prof_run.log" 2>&1 || exit $?
cd "$R"; S=$(find "$O/prof" -name "*kernel_stats.csv" | head -n1)
python scripts/summarize_prof.py "$S" 9 "ViT kernel stats ($TAG)" > "$O/kernel_stats.md" 2>&1; head -24 "$O/kernel_stats.md"
exit 0
