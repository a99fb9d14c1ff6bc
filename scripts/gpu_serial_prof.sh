#!/bin/bash
# Serialized-step profile (weight-gradient side stream off): per-kernel costs without stream overlap.
# Usage: gpurun -- bash scripts/gpu_serial_prof.sh <tag> [bench args...]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
TAG="${1:-serial}"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export PVR_SIDE_WGRAD=0
timeout -k 10 240 python bench.py "$@" > "$O/bench_serial.log" 2>&1 || exit $?
tail -1 "$O/bench_serial.log" | cut -c1-200
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 3 "$@" > "$O/prof_run.log" 2>&1 || exit $?
cd "$R"; S=$(find "$O/prof" -name "*kernel_stats.csv" | head -n1)
python scripts/summarize_prof.py "$S" 9 "ViT kernel stats, serialized ($TAG)" > "$O/kernel_stats.md" 2>&1; head -30 "$O/kernel_stats.md"
exit 0
