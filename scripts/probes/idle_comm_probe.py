"""Does an idle second RCCL communicator slow the GPU? (native-transport world-1 deficit)

Times the ViT-B/16 b256 eval forward (memory- and MFMA-bound kernels, no collectives) in three
states of one process: (a) world-1 torch.distributed group only, (b) + a torch RCCL communicator
(first collective), (c) + the framework's native RCCL communicator (parallel/comm.py). Prints
ms per forward for each state.

Run: python scripts/probes/idle_comm_probe.py (one GPU).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.distributed as dist


def timed(model, x, n=30):
    with torch.inference_mode():
        for _ in range(5):
            model(x)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            model(x)
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from pytorch_vit_paper_replication_amd.models import ViT

    model = ViT().cuda().eval()
    x = torch.rand(256, 3, 224, 224, device="cuda")
    print(f"pg only        : {timed(model, x):.3f} ms", flush=True)
    t = torch.ones(1, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"+ torch comm   : {timed(model, x):.3f} ms", flush=True)
    from pytorch_vit_paper_replication_amd.parallel.comm import NativeCommunicator

    c = NativeCommunicator.create(torch.device("cuda", 0))
    c.wait(c.all_reduce(t))
    torch.cuda.synchronize()
    print(f"+ native comm  : {timed(model, x):.3f} ms", flush=True)
    print(f"again          : {timed(model, x):.3f} ms", flush=True)
    c.destroy()
    torch.cuda.synchronize()
    print(f"native destroyed: {timed(model, x):.3f} ms", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
