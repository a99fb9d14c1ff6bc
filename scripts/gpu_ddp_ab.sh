#!/bin/bash
# b512 step: no process group / world-1 process group only / DDP over torch.distributed / DDP over
# the native RCCL communicator (why is the world-1 DDP run slower, and where).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ddpab
for v in "plain:" "pg:--pg-only" "ddp_torch:--force-ddp --comm torch" "ddp_native:--force-ddp --comm native" "plain2:"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python bench.py --steps 8 --warmup 3 --batch 512 $a > gpurun_out/ddpab/$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(tail -1 gpurun_out/ddpab/$n.log | cut -c 90-160)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
