#!/bin/bash
# Serving: eager vs hipGraph-replayed eval forward at small batches; reference-style PyTorch (autocast bf16) at b256.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/infer2; mkdir -p $O; export TMPDIR=/tmp
for args in "--batch 1" "--batch 1 --graph" "--batch 8" "--batch 8 --graph" "--batch 32" "--batch 32 --graph" "--batch 256 --graph" "--batch 256 --impl torch"; do
  timeout -k 10 300 python bench.py --infer --steps 50 --warmup 10 $args > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "infer $args: $(tail -1 $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms")')"
done
