#!/bin/bash
# Round 5, verdict item 8: side-stream weight gradients vs serial, alternated inside one session on
# B/16 (bf16, b256) and H/14 (fp8 default, b256); then the steady-state step tables of the three
# BASELINE configs (kernel trace of the serial schedule -> scripts/steady_step.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5side}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
prof() {
  local n=$1 title=$2; shift 2
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/${n}_prof" -o step --output-format csv -- python3 "$R/bench.py" "$@" --serial-wgrad > "$R/$O/${n}_prof.log" 2>&1; local rc=$?
  cd "$R"; echo "[$n prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/steady_step.py "$(find "$O/${n}_prof" -name "*kernel_trace.csv" | head -n1)" "$title" > "$O/${n}_steady.md"
  rm -rf "$O/${n}_prof"
  head -n 3 "$O/${n}_steady.md" | tail -n 1
}
for i in 1 2 3; do
  step 200 b16_side_$i.log python bench.py
  step 200 b16_serial_$i.log python bench.py --serial-wgrad
done
step 200 b16b512_side.log python bench.py --batch 512 --steps 10 --warmup 3
step 200 b16b512_serial.log python bench.py --batch 512 --steps 10 --warmup 3 --serial-wgrad
for i in 1 2; do
  step 300 h14_side_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
  step 300 h14_serial_$i.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4 --serial-wgrad
done
prof b16 "ViT-B/16 b256 bf16" --steps 3 --warmup 2
prof h14 "ViT-H/14 b256 fp8 (bf16 wgrad)" --model vit_h14 --dtype fp8 --steps 3 --warmup 2
prof l16 "ViT-L/16@384 b128 bf16" --model vit_l16 --image-size 384 --steps 3 --warmup 2
