#!/bin/bash
# One-off probe session: runs the python script named in $PROBE (with $PROBE_ARGS) under a time limit.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PROBE_T:-300} python -u $PROBE $PROBE_ARGS > gpurun_out/probe.log 2>&1
rc=$?
tail -n 40 gpurun_out/probe.log | cut -c1-600
exit $rc
