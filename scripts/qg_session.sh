#!/bin/bash
# GPU session: attention forward query-group / key-tile A/B after the staged output
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/qg; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/attn_ab.py --ab fwd_qg --shapes h14,l16_384 > gpurun_out/qg/attn_ab_fwd_qg.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/qg/attn_ab_fwd_qg.log; exit $rc
