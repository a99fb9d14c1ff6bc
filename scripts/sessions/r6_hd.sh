#!/bin/bash
# Round 6: headline bench alternating the working tree (PVR_DROP_MASK=0) with an A/B tree (abv/<name>),
# then the A/B tree's steady-state table.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-hd}; mkdir -p "$O"; V=${2:-head}
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
for r in 1 2 3; do
  PVR_PKG_ROOT=abv/$V run 240 ${V}_$r.log python bench.py --steps 30 --warmup 5
  PVR_DROP_MASK=0 run 240 wt_$r.log python bench.py --steps 30 --warmup 5
done
export PVR_PKG_ROOT=abv/$V
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/${V}_prof" -o step --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --serial-wgrad > "$R/$O/${V}_prof.log" 2>&1 || exit $?
cd "$R"; python scripts/steady_step.py "$(find "$O/${V}_prof" -name "*kernel_trace.csv" | head -n1)" "ViT-B/16 b256 bf16 ($V)" > "$O/${V}_steady.md"
rm -rf "$O/${V}_prof"; grep -v "^$" "$O/${V}_steady.md" | head -8
