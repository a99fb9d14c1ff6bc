#!/bin/bash
# Same-box check + A/B for the dq tail-mask change: GPU tests and attention kbench on this tree,
# then the headline bench alternating this tree and ab_base (the previous commit, built).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/abm; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/abm/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/abm/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "new:$R" "old:$R/ab_base"; do
  n=${v%%:*}; d=${v#*:}
  (cd "$d" && timeout -k 10 120 python scripts/bench_kernels.py --only attn) > gpurun_out/abm/kb_$n.log 2>&1
  rc=$?; echo "kb_$n rc=$rc"; grep attn_ gpurun_out/abm/kb_$n.log; [ $rc -ne 0 ] && exit $rc
done
AB_TREE=ab_base bash scripts/gpu_ab_tree.sh
