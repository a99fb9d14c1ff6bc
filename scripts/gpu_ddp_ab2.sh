#!/bin/bash
# World-1 DDP transports A/B after resolving RCCL from torch's own library.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/ddpab
timeout -k 10 60 python -c "import torch; from pytorch_vit_paper_replication_amd import _ext; e=_ext.ext(); print('rccl', e.rccl_version(), e.rccl_path())" 2>&1 | tail -1
for v in "ddp_native:--force-ddp --comm native" "ddp_torch:--force-ddp --comm torch" "ddp_native2:--force-ddp --comm native" "plain:"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python bench.py --steps 8 --warmup 3 --batch 512 $a > gpurun_out/ddpab/$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ddpab/$n.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
