#!/bin/bash
# rocprofv3 counter passes over the ViT-H/14 fp8 GEMMs and torch._scaled_mm on the same operands
# (scripts/fp8_vs_scaled_mm.py, one round) or, with a second argument "b16", over the ViT-B/16 bf16
# GEMMs and torch.matmul (scripts/gemm_ab.py); one pass per counter set, each under its own timeout.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${1:-pmc_gemm}"; mkdir -p "$O"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
PROG=fp8_vs_scaled_mm.py
[ "${2:-}" = "b16" ] && PROG=gemm_ab.py
cd /tmp
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d "$O/p$i" -o run --output-format csv -- python3 "$R/scripts/$PROG" --rounds 1 > "$O/p$i.log" 2>&1
  rc=$?; echo "[pmc pass $i] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$R" && python3 scripts/pmc_summary.py "$O" "gemm|Cijk|scaled|splitk" > "$O/summary.md" && echo "[pmc summary] ok"
