#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out/pmc_attn"; export TMPDIR=/tmp; cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d "$R/gpurun_out/pmc_attn" -o set$i --output-format csv -- python3 "$R/scripts/attn_probe.py" > "$R/gpurun_out/pmc_attn/set$i.log" 2>&1
  rc=$?; echo "set$i rc=$rc"; tail -3 "$R/gpurun_out/pmc_attn/set$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
ls "$R/gpurun_out/pmc_attn"
