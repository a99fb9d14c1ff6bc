#!/bin/bash
# Patch-embedding GEMM on the LDS-staged epilogue: checks, kernel time, step.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/pe; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 180 python scripts/run_checks.py check_gemm_patch_embed_epilogue,check_vit_fused_vs_reference,check_vit_block_link,check_patch_bwd,check_vit_inference > $O/checks.log 2>&1; rc=$?
grep -v amdgpu.ids $O/checks.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o k --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 2 > "$R/$O/prof.log" 2>&1 || exit $?
cd "$R"; S=$(find "$O/prof" -name "*kernel_stats.csv" | head -n1); python3 scripts/summarize_prof.py "$S" 6 "pe" > $O/ks.md; grep -E "gemm_pp_kernel<true, true, true, 0|im2col|cls_rows" $O/ks.md
python3 - "$R/$O/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("void pvr::(anonymous namespace)::gemm_pp_kernel<true, true, true, 0") and r["Grid_Size_X"] == "301056"]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("patch-embed GEMM (grid 301056) us per call:", [round(x, 1) for x in d])
PY
for i in 1 2; do timeout -k 10 300 python bench.py > $O/b.log 2>&1 || exit $?; tail -1 $O/b.log | cut -c1-150; done
