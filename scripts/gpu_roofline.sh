#!/bin/bash
# Roofline evidence for the ViT-B/16 b256 step with the side stream off (clean per-kernel times):
# kernel trace + stats, then one PMC pass each for HBM read bytes, HBM write bytes and MFMA busy cycles.
R="${GRAFT_REPO_ROOT:-/root/repo}"; O="$R/gpurun_out/roof"; mkdir -p "$O"; export TMPDIR=/tmp; cd /tmp
export PVR_SIDE_WGRAD=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o k --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 > "$O/trace.log" 2>&1 || exit $?
tail -1 "$O/trace.log" | cut -c1-160
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set -d "$O/pmc$i" -o p --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$O/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($set) rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/pmc$i.log"; exit $rc; }
done
ls -R "$O" | head -40
