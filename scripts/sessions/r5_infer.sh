#!/bin/bash
# Round 5: serving throughput / latency refresh (bench.py --infer: eval forward under inference_mode),
# the round-2 table's rows with the round-5 kernels.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5infer}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; }
step 200 b256.log python bench.py --infer --batch 256 --steps 30 --warmup 5
step 200 b256_graph.log python bench.py --infer --batch 256 --graph --steps 30 --warmup 5
step 200 b1024.log python bench.py --infer --batch 1024 --steps 20 --warmup 5
step 200 b1.log python bench.py --infer --batch 1 --steps 100 --warmup 10
step 200 b8.log python bench.py --infer --batch 8 --steps 100 --warmup 10
step 200 b32.log python bench.py --infer --batch 32 --steps 50 --warmup 10
step 300 l16_384_b128.log python bench.py --infer --model vit_l16 --image-size 384 --batch 128 --steps 20 --warmup 5
step 300 h14_b256.log python bench.py --infer --model vit_h14 --batch 256 --steps 20 --warmup 5
step 300 b256_torch.log python bench.py --infer --batch 256 --impl torch --steps 20 --warmup 5
