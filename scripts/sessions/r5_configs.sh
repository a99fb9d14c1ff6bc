#!/bin/bash
# Round 5: BASELINE configs 3-5 at their per-GPU batch on one GPU, wrapped in DDP (--force-ddp: the
# world-1 RCCL process group, bucketed all-reduce hooks and all): img/s and peak memory per GPU, and the
# fp8 weight-gradient opt-in next to the (new) bf16-wgrad fp8 default.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r5configs; mkdir -p $O; export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -n1 $O/$log | cut -c1-400; [ $rc -eq 0 ] || { tail -5 $O/$log; exit $rc; }; }
run 300 b16_b512_ddp.log python bench.py --batch 512 --force-ddp --steps 20 --warmup 5
run 300 b16_b256.log python bench.py --steps 20 --warmup 5
run 400 l16_384_b128_ddp.log python bench.py --model vit_l16 --image-size 384 --force-ddp --steps 10 --warmup 4
run 500 h14_fp8_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --force-ddp --steps 8 --warmup 4
run 500 h14_fp8w_b256.log python bench.py --model vit_h14 --dtype fp8 --fp8-wgrad --steps 8 --warmup 4
run 500 h14_fp8_b256.log python bench.py --model vit_h14 --dtype fp8 --steps 8 --warmup 4
