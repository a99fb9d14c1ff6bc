#!/bin/bash
# Round 6 verification: the GPU test suite (with the 2-rank gloo bench test) and smoke, then the
# hipGraph question (eager vs --serial-wgrad vs --main-prio 0 vs --graph, ViT-B/16 b256) and a
# world-1 RCCL DDP run at b512 with per-bucket all-reduce times.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-v1}; mkdir -p "$O"; PART=${2:-all}
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
if [ "$PART" = all ] || [ "$PART" = tests ]; then
  run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  grep -E "passed|failed" "$O/pytest_gpu.log" | tail -n 2
  run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
fi
if [ "$PART" = all ] || [ "$PART" = bench ]; then
  for r in 1 2; do
    run 240 eager_$r.log python bench.py --steps 30 --warmup 5
    run 240 serialwg_$r.log python bench.py --steps 30 --warmup 5 --serial-wgrad
    run 240 prio0_$r.log python bench.py --steps 30 --warmup 5 --main-prio 0
    run 300 graph_$r.log python bench.py --steps 30 --warmup 5 --graph
  done
  run 400 ddp_w1_b512.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --batch 512 --force-ddp --steps 20 --warmup 5 --metrics-jsonl "$O/ddp_w1_b512.jsonl"
fi
