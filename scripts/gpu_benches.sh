#!/bin/bash
# pytest -m gpu, smoke, benches: B/16 b256 (headline), b512 DDP world 1 (the per-GPU config of the
# multi-GPU runs), L/16@384, H/14 bf16 and fp8.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-1} "$R/gpurun_out/$log" | cut -c1-330
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=3 run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 180 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench.log python bench.py --steps 20 --warmup 5
run 300 bench_b512_ddp.log python bench.py --steps 10 --warmup 3 --batch 512 --force-ddp
run 300 bench_l16_384.log python bench.py --model vit_l16 --image-size 384 --batch 64 --steps 5 --warmup 2
run 300 bench_h14.log python bench.py --model vit_h14 --batch 128 --steps 5 --warmup 2
run 300 bench_h14_fp8.log python bench.py --model vit_h14 --batch 128 --steps 5 --warmup 2 --dtype fp8
exit 0
