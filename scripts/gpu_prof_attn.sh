#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out/pattn"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pattn" -o tr --output-format csv -- python3 "$R/scripts/attn_probe.py" > "$R/gpurun_out/pattn/tr.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$R/gpurun_out/pattn" -o p1 --output-format csv -- python3 "$R/scripts/attn_probe.py" > "$R/gpurun_out/pattn/p1.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d "$R/gpurun_out/pattn" -o p2 --output-format csv -- python3 "$R/scripts/attn_probe.py" > "$R/gpurun_out/pattn/p2.log" 2>&1 || exit $?
echo ok
