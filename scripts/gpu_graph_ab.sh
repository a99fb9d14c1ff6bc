#!/bin/bash
# hipGraph replay of the whole step vs eager launches, with and without the weight-gradient side stream.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/graph; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag env... -- bench args
  local tag="$1"; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 $BARGS > $O/$tag.log 2>&1 || return $?
  echo "$tag $BARGS $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["impl"])')"
}
for b in 32 256; do
  export BARGS="--batch $b"
  run eager_b$b PVR_SIDE_WGRAD=1 || exit $?
  run eager_serial_b$b PVR_SIDE_WGRAD=0 || exit $?
  BARGS="--batch $b --graph" run graph_b$b PVR_SIDE_WGRAD=1 || exit $?
  BARGS="--batch $b --graph" run graph_serial_b$b PVR_SIDE_WGRAD=0 || exit $?
done
