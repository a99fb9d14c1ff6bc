mkdir -p gpurun_out/det
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/det/kernels.log 2>&1; rc=$?
grep "deterministic ordered\|passed\|failed" gpurun_out/det/kernels.log | cut -c1-250
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/sessions/r6_e4m3_study.sh e4m3_study 0
