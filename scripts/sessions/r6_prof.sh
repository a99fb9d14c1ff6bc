#!/bin/bash
# Round 6: steady-state step tables (rocprofv3 kernel trace, serial weight gradients) of ViT-B/16
# b256 for the variants given as NAME=ENVVAR=VALUE arguments ("main" = no override).
#   gpurun -- bash scripts/sessions/r6_prof.sh <tag> main dmoff=PVR_DROP_MASK=0
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${1:-prof}; mkdir -p "$O"; shift
for v in "$@"; do
  n=${v%%=*}; kv=${v#*=}
  (
    if [ "$kv" != "$v" ]; then export "$kv"; fi
    cd /tmp
    timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/$O/${n}_prof" -o step --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --serial-wgrad > "$R/$O/${n}_prof.log" 2>&1
  ); rc=$?
  echo "[$n prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/steady_step.py "$(find "$O/${n}_prof" -name "*kernel_trace.csv" | head -n1)" "ViT-B/16 b256 bf16 ($v)" > "$O/${n}_steady.md"
  rm -rf "$O/${n}_prof"
  head -n 3 "$O/${n}_steady.md" | tail -n 1
done
