#!/bin/bash
# Kernel-time profiles of the BASELINE configs: ViT-B/16 224 px bf16 (b256, headline), ViT-L/16 384 px bf16 (b64),
# ViT-H/14 224 px fp8 (b128).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${1:-models}"; mkdir -p "$O"
run() {  # tag, bench args...
  local tag="$1"; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 "$@" > "$O/bench_$tag.log" 2>&1 || return $?
  tail -1 "$O/bench_$tag.log" | cut -c1-220
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$tag" -o k --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 2 "$@" > "$O/prof_$tag.log" 2>&1 || return $?
  cd "$R"; S=$(find "$O/prof_$tag" -name "*kernel_stats.csv" | head -n1)
  python scripts/summarize_prof.py "$S" 6 "kernel stats $tag" > "$O/kernel_stats_$tag.md" 2>&1; head -20 "$O/kernel_stats_$tag.md"
}
run b16_b256 || exit $?
run l16_384 --model vit_l16 --image-size 384 --batch 64 || exit $?
run h14_fp8 --model vit_h14 --batch 128 --dtype fp8 || exit $?
exit 0
