#!/bin/bash
# DDP transports at world 1 vs no DDP (same box, back to back), per-step JSONL, native-transport profile.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ddp; export TMPDIR=/tmp
B="timeout -k 10 240 python bench.py --steps 30 --warmup 5 --batch 512"
$B > gpurun_out/ddp/none.log 2>&1 && tail -1 gpurun_out/ddp/none.log | cut -c1-150 &&
$B --force-ddp --metrics-jsonl gpurun_out/ddp/steps_torch.jsonl > gpurun_out/ddp/torch.log 2>&1 && tail -1 gpurun_out/ddp/torch.log | cut -c1-150 &&
$B --force-ddp --comm-dtype bf16 > gpurun_out/ddp/torch_bf16.log 2>&1 && tail -1 gpurun_out/ddp/torch_bf16.log | cut -c1-150 &&
$B --force-ddp --comm native > gpurun_out/ddp/native.log 2>&1 && tail -1 gpurun_out/ddp/native.log | cut -c1-150 &&
$B > gpurun_out/ddp/none2.log 2>&1 && tail -1 gpurun_out/ddp/none2.log | cut -c1-150 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ddp/prof_native -o native -- python bench.py --steps 10 --warmup 3 --batch 512 --force-ddp --comm native > gpurun_out/ddp/prof_native.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ddp/prof_torch -o torch -- python bench.py --steps 10 --warmup 3 --batch 512 --force-ddp > gpurun_out/ddp/prof_torch.log 2>&1 &&
echo profiled
