#!/bin/bash
# Round 5, final: the round-end checks (GPU suite, smoke), the headline bench, the BASELINE configs
# at their per-GPU batch (DDP world 1), and the steady-state step tables (serial schedule).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5final}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|peak_mem_gb": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; }
prof() {
  local n=$1 title=$2; shift 2
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/${n}_prof" -o step --output-format csv -- python3 "$R/bench.py" "$@" --serial-wgrad > "$R/$O/${n}_prof.log" 2>&1; local rc=$?
  cd "$R"; echo "[$n prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/steady_step.py "$(find "$O/${n}_prof" -name "*kernel_trace.csv" | head -n1)" "$title" > "$O/${n}_steady.md"
  rm -rf "$O/${n}_prof"
  head -n 3 "$O/${n}_steady.md" | tail -n 1
}
step 1100 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step 200 b16_$i.log python bench.py; done
step 300 b16_b512_ddp.log python bench.py --batch 512 --force-ddp --steps 20 --warmup 5
step 400 l16_384_b128_ddp.log python bench.py --model vit_l16 --image-size 384 --force-ddp --steps 10 --warmup 4
step 500 h14_fp8_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --force-ddp --steps 8 --warmup 4
step 500 h14_fp8w_b256.log python bench.py --model vit_h14 --dtype fp8 --fp8-wgrad --steps 8 --warmup 4
prof b16 "ViT-B/16 b256 bf16" --steps 3 --warmup 2
prof h14 "ViT-H/14 b256 fp8 (bf16 wgrad)" --model vit_h14 --dtype fp8 --steps 3 --warmup 2
prof l16 "ViT-L/16@384 b128 bf16" --model vit_l16 --image-size 384 --steps 3 --warmup 2
