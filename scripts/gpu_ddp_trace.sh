#!/bin/bash
# Kernel traces of the b512 step with and without the DDP wrapper (world 1): where the DDP
# overhead goes (RCCL kernels, stream gaps).
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out/ddptr"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ddptr" -o ddp --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 2 --batch 512 --force-ddp > "$R/gpurun_out/ddptr/ddp.log" 2>&1
rc=$?; echo "ddp rc=$rc"; tail -1 "$R/gpurun_out/ddptr/ddp.log" | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ddptr" -o plain --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 2 --batch 512 > "$R/gpurun_out/ddptr/plain.log" 2>&1
rc=$?; echo "plain rc=$rc"; tail -1 "$R/gpurun_out/ddptr/plain.log" | cut -c1-200
exit $rc
