#!/bin/bash
# Round 6: in-launch split-K reduction of the weight gradients: checks, wgrad timings on / off, then
# the headline bench alternating PVR_SPLITK_FIXUP=1 / 0, and one serial-wgrad rocprofv3 stats run.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-sk1}; mkdir -p "$O"
run() { local t=$1 log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(grep -o '"value": [0-9.]*' "$O/$log" | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -n 30 "$O/$log"; exit $rc; }; }
run 300 checks.log python -u scripts/run_checks.py check_gemm_wgrad
cat "$O/checks.log"
run 300 wgrad_ab.log python scripts/gemm_ab.py --ab skfix --only wgrad
grep "ours\|hipBLASLt" "$O/wgrad_ab.log"
for r in 1 2 3; do
  run 240 on_$r.log python bench.py --steps 30 --warmup 5
  PVR_SPLITK_FIXUP=0 run 240 off_$r.log python bench.py --steps 30 --warmup 5
done
run 300 ser_on.log python bench.py --steps 30 --warmup 5 --serial-wgrad
PVR_SPLITK_FIXUP=0 run 300 ser_off.log python bench.py --steps 30 --warmup 5 --serial-wgrad
