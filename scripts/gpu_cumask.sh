#!/bin/bash
# Weight-gradient side stream confined to a CU partition (hipExtStreamCreateWithCUMask) vs the
# unrestricted side stream, same box, alternating.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/cumask
for i in 1 2; do
  for v in "none:" "c128:0-127" "m2:mod:2:0" "c160:0-159" "m8x5:mod:8:0+1+2+3+4"; do
    n=${v%%:*}; m=${v#*:}
    PVR_SIDE_CU_MASK="$m" timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/cumask/$n$i.log 2>&1
    rc=$?; echo "$n ($m) rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/cumask/$n$i.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
