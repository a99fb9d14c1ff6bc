#!/bin/bash
# GPU session: bf16 persistent GEMM K limit A/B on ViT-L/16@384 b128 and ViT-B/16 b256
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-pmaxk}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 1 "$O/$log" | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
for k in 0 2048 0 2048; do
  a=""; [ "$k" != "0" ] && a="--persistent-max-k $k"
  step 300 l16_k$k.log python bench.py --model vit_l16 --image-size 384 --batch 128 --steps 6 --warmup 3 $a
done
for k in 0 1024 0 1024; do
  a=""; [ "$k" != "0" ] && a="--persistent-max-k $k"
  step 200 b16_k$k.log python bench.py $a
done
