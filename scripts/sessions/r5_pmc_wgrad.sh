#!/bin/bash
# Round 5: why the weight-gradient GEMM (mn-contiguous operands) runs at ~50 % of the MFMA rate while
# the k-contiguous forward reaches ~75 %: PMC passes over the qkv wgrad and the qkv forward (separate
# processes), each counter set in its own run.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/${1:-r5pmcw}; mkdir -p "$O"
step() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "[$log] rc=$rc"; tail -n 2 "$O/$log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step 120 time_wgrad.log python scripts/gemm_pmc_probe.py --kind wgrad --iters 20
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for k in wgrad fwd; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    cd /tmp
    timeout -s KILL 90 rocprofv3 --pmc $P -d "$R/$O/${k}_p$i" -o pmc --output-format csv -- python3 "$R/scripts/gemm_pmc_probe.py" --kind $k --iters 6 > "$R/$O/${k}_p$i.log" 2>&1; rc=$?
    cd "$R"; echo "[$k p$i] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
