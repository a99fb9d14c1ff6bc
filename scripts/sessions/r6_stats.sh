#!/bin/bash
# Round 6, last tree: rocprofv3 --kernel-trace --stats of the default headline bench (side stream on)
# and of the ViT-H/14 fp8 bench; the per-kernel stats CSVs are kept.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-stats}; mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/b16" -o b16 --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/$O/b16.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/h14" -o h14 --output-format csv -- python3 "$R/bench.py" --model vit_h14 --dtype fp8 --steps 4 --warmup 3 > "$R/$O/h14.log" 2>&1 || exit $?
cd "$R"
for n in b16 h14; do
  f=$(find "$O/$n" -name "*kernel_stats.csv" | head -n1); cp "$f" "$O/${n}_kernel_stats.csv"; rm -rf "$O/$n"
  head -n 12 "$O/${n}_kernel_stats.csv" | cut -c1-160
done
