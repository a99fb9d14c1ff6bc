#!/bin/bash
# Round 6: the BASELINE configs at their per-GPU batch (DDP world 1) and the steady-state step tables
# of ViT-L/16-384 and ViT-H/14 fp8 (serial weight gradients).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-configs}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|peak_mem_gb": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
prof() {
  local n=$1 title=$2; shift 2
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/${n}_prof" -o step --output-format csv -- python3 "$R/bench.py" "$@" --serial-wgrad > "$R/$O/${n}_prof.log" 2>&1; local rc=$?
  cd "$R"; echo "[$n prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/steady_step.py "$(find "$O/${n}_prof" -name "*kernel_trace.csv" | head -n1)" "$title" > "$O/${n}_steady.md"
  rm -rf "$O/${n}_prof"
  head -n 3 "$O/${n}_steady.md" | tail -n 1
}
run 400 l16_384_b128_ddp.log python bench.py --model vit_l16 --image-size 384 --force-ddp --steps 10 --warmup 4
run 500 h14_fp8_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --force-ddp --steps 8 --warmup 4
run 500 h14_fp8_bf16wgrad_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --fp8-bf16-wgrad --force-ddp --steps 8 --warmup 4
run 500 h14_bf16_b256_ddp.log python bench.py --model vit_h14 --force-ddp --steps 8 --warmup 4
prof h14 "ViT-H/14 b256 fp8 (fp8 wgrad)" --model vit_h14 --dtype fp8 --steps 3 --warmup 2
prof l16 "ViT-L/16@384 b128 bf16" --model vit_l16 --image-size 384 --steps 3 --warmup 2
