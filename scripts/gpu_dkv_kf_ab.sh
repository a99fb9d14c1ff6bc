#!/bin/bash
# dK/dV backward: 16 keys per wave (PVR_DKV_KF=1, 13 waves at N = 197) vs 32 (KF=2, 7 waves).
# GPU tests under KF=1, then attention kbench and the headline bench alternating both, one box.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/kf; export TMPDIR=/tmp
PVR_DKV_KF=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/kf/pytest_kf1.log 2>&1
rc=$?; echo "pytest kf1 rc=$rc"; tail -2 gpurun_out/kf/pytest_kf1.log; [ $rc -ne 0 ] && exit $rc
for kf in 1 2; do
  PVR_DKV_KF=$kf timeout -k 10 120 python scripts/bench_kernels.py --only attn > gpurun_out/kf/kb_$kf.log 2>&1
  rc=$?; echo "kb kf$kf rc=$rc"; grep attn_bwd gpurun_out/kf/kb_$kf.log; [ $rc -ne 0 ] && exit $rc
done
for i in 1 2 3; do
  for kf in 1 2; do
    PVR_DKV_KF=$kf timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/kf/b_${kf}_$i.log 2>&1
    rc=$?; echo "bench kf$kf #$i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/kf/b_${kf}_$i.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
