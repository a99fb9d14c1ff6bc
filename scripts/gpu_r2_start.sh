#!/bin/bash
# Session start check: GPU test tier, smoke, headline bench, in-step kernel stats.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; O=gpurun_out/r2s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log && \
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-300 && \
timeout -k 10 200 python bench.py --batch 512 --force-ddp > $O/bench_ddp512.log 2>&1 && tail -1 $O/bench_ddp512.log | cut -c1-300
