#!/bin/bash
# Kernel trace of the headline bench + PMC counter passes over the attention kernels.
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out/prof3" "$R/gpurun_out/pmc3"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof3" -o vitb16 --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 3 > "$R/gpurun_out/prof3/run.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 "$R/gpurun_out/prof3/run.log" | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d "$R/gpurun_out/pmc3" -o set$i --output-format csv -- python3 "$R/scripts/attn_probe.py" > "$R/gpurun_out/pmc3/set$i.log" 2>&1
  rc=$?; echo "set$i rc=$rc"; tail -1 "$R/gpurun_out/pmc3/set$i.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
