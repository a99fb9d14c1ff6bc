#!/bin/bash
# Round 6, final tree (e4m3 fp8 gradients by default, deterministic attention slabs): GPU suite, smoke,
# headline bench x3, world-1 RCCL b512, the BASELINE configs at their per-GPU batch, B/16 steady table.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-verify3}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed\|[0-9]* failed\|peak_mem_gb": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2 3; do run 240 b16_$i.log python bench.py; done
run 400 b16_b512_ddp.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --batch 512 --force-ddp --steps 20 --warmup 5
run 500 h14_fp8_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --force-ddp --steps 8 --warmup 4
run 500 h14_fp8_e5m2_b256_ddp.log python bench.py --model vit_h14 --dtype fp8 --fp8-grad e5m2 --force-ddp --steps 8 --warmup 4
run 400 l16_384_b128_ddp.log python bench.py --model vit_l16 --image-size 384 --force-ddp --steps 10 --warmup 4
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/b16_prof" -o step --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --serial-wgrad > "$R/$O/b16_prof.log" 2>&1 || exit $?
cd "$R"; python scripts/steady_step.py "$(find "$O/b16_prof" -name "*kernel_trace.csv" | head -n1)" "ViT-B/16 b256 bf16" > "$O/b16_steady.md"
rm -rf "$O/b16_prof"; grep -v "^$" "$O/b16_steady.md" | head -6
