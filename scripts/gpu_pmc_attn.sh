#!/bin/bash
# PMC counter passes over the attention kernels (one rocprofv3 run per counter set).
# usage: gpu_pmc_attn.sh [fwd|bwd|both] [outdir-name]
R="${GRAFT_REPO_ROOT:-/root/repo}"; W="${1:-both}"; O="$R/gpurun_out/${2:-pmc_attn}"; mkdir -p "$O"; export TMPDIR=/tmp; cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d "$O" -o set$i --output-format csv -- python3 "$R/scripts/attn_probe.py" $W > "$O/set$i.log" 2>&1
  rc=$?; echo "set$i rc=$rc"; tail -1 "$O/set$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
