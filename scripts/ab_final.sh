#!/bin/bash
# Round-4 evidence session: full GPU test suite, smoke, BASELINE benches, serial-wgrad step profiles.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-final}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
prof() {  # prof <name> <bench args...>: serial-wgrad kernel trace + stats summary
  local n=$1; shift
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/${n}_prof" -o step --output-format csv -- python3 "$R/bench.py" "$@" --serial-wgrad > "$R/$O/${n}_prof.log" 2>&1; local rc=$?
  cd "$R"; echo "[$n prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  local S; S=$(find "$O/${n}_prof" -name "*kernel_stats.csv" | head -n1)
  python scripts/summarize_prof.py "$S" 7 "$n kernel stats (r4 final, serial wgrad)" > "$O/${n}_kernel_stats_serial.md" 2>&1
}
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 200 b_def.log python bench.py
step 300 h14_def.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
step 300 l16_def.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 6 --warmup 3
prof h14 --model vit_h14 --dtype fp8 --batch 256 --steps 4 --warmup 3
prof l16 --model vit_l16 --image-size 384 --batch 128 --steps 3 --warmup 2
prof b16 --steps 4 --warmup 3
