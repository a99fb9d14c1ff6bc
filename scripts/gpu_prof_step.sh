#!/bin/bash
# Kernel trace of the headline bench step: in-step (side stream on) and serialized (PVR_SIDE_WGRAD=0)
# kernel statistics + the step timeline. Usage: gpurun -- bash scripts/gpu_prof_step.sh <tag> [bench args]
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
TAG="${1:-prof}"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
for mode in instep serial; do
  if [ $mode = serial ]; then export PVR_SIDE_WGRAD=0; fi
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$mode" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 3 "$@" > "$O/${mode}_run.log" 2>&1
  rc=$?; cd "$R"
  if [ $rc -ne 0 ]; then echo "STOP $mode rc=$rc"; tail -5 "$O/${mode}_run.log"; exit $rc; fi
  tail -1 "$O/${mode}_run.log" | cut -c1-160
  S=$(find "$O/$mode" -name "*kernel_stats.csv" | head -n1)
  T=$(find "$O/$mode" -name "*kernel_trace.csv" | head -n1)
  python scripts/summarize_prof.py "$S" 9 "ViT-B/16 b256 kernel stats ($TAG, $mode)" > "$O/kernel_stats_$mode.md" 2>&1
  python scripts/step_timeline.py "$T" > "$O/timeline_$mode.txt" 2>&1
  head -3 "$O/timeline_$mode.txt"; sed -n '5,30p' "$O/kernel_stats_$mode.md" | cut -c1-150
done
exit 0
