#!/bin/bash
# Same-box A/B of the headline bench between this tree and a second built tree (AB_TREE, e.g. a git
# worktree of an older commit), alternating so box drift cancels out.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/abtree
OLD="$R/${AB_TREE:-ab_old}"
for i in 1 2 3; do
  for v in "new:$R" "old:$OLD"; do
    n=${v%%:*}; d=${v#*:}
    (cd "$d" && timeout -k 10 200 python bench.py --steps 15 --warmup 4 ${BENCH_ARGS}) > gpurun_out/abtree/$n$i.log 2>&1
    rc=$?; echo "$n$i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/abtree/$n$i.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
