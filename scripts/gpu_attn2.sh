#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/pmc4
run() {
  local t=$1; local log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n ${TAILN:-2} "$R/gpurun_out/$log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
  return 0
}
TAILN=3 run 400 checks.log python tests/kernel_checks.py
TAILN=3 run 200 kb_attn.log python scripts/bench_kernels.py --only attn
run 300 bench.log python bench.py --steps 20 --warmup 5
export TMPDIR=/tmp
cd /tmp
TAILN=1 run 120 pmc4/set1.log rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc4" -o set1 --output-format csv -- python3 "$R/scripts/attn_probe.py"
TAILN=1 run 120 pmc4/set2.log rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d "$R/gpurun_out/pmc4" -o set2 --output-format csv -- python3 "$R/scripts/attn_probe.py"
exit 0
