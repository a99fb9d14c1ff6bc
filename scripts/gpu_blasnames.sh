#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/blas"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/blas" -o blas --output-format csv -- python3 "$R/scripts/blas_names.py" > "$R/gpurun_out/blas.log" 2>&1
echo rc=$?
