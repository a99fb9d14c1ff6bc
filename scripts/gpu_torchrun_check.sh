cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/tr
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 --force-ddp > gpurun_out/tr/torchrun_ddp_w1.log 2>&1 && tail -1 gpurun_out/tr/torchrun_ddp_w1.log | cut -c1-420 && \
timeout -k 10 300 python bench.py --model vit_h14 --batch 128 --dtype fp8 --steps 8 --warmup 3 > gpurun_out/tr/h14_fp8.log 2>&1 && tail -1 gpurun_out/tr/h14_fp8.log | cut -c1-300
