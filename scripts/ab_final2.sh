#!/bin/bash
# Round-4 closing evidence: full GPU suite, smoke, BASELINE benches, steady-state step tables.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-final2}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
prof() {  # prof <name> <title> <bench args...>: serial-wgrad kernel trace -> one steady-state step table
  local n=$1 title=$2; shift 2
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/${n}_prof" -o step --output-format csv -- python3 "$R/bench.py" "$@" --serial-wgrad > "$R/$O/${n}_prof.log" 2>&1; local rc=$?
  cd "$R"; echo "[$n prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/steady_step.py "$(find "$O/${n}_prof" -name "*kernel_trace.csv" | head -n1)" "$title" > "$O/${n}_steady.md"
  rm -rf "$O/${n}_prof"
  head -n 3 "$O/${n}_steady.md" | tail -n 1
}
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 200 b_def.log python bench.py
step 200 b_def2.log python bench.py
step 300 h14_def.log python bench.py --model vit_h14 --dtype fp8 --batch 256 --steps 8 --warmup 4
step 300 l16_def.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 6 --warmup 3
prof b16 "ViT-B/16 b256 bf16" --steps 3 --warmup 2
prof h14 "ViT-H/14 b256 fp8" --model vit_h14 --dtype fp8 --batch 256 --steps 3 --warmup 2
prof l16 "ViT-L/16@384 b128 bf16" --model vit_l16 --image-size 384 --batch 128 --steps 3 --warmup 2
