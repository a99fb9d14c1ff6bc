#!/usr/bin/env python3
"""Headline benchmark: training images/sec for ViT-B/16 @224 px, bf16, on 1..8 MI355X (BASELINE.json).

One process per GPU (``torch.distributed.run``), RCCL gradient all-reduce via the framework's
bucketed DDP. Each step is a full training step of the reference recipe: forward, mean
cross-entropy, backward, global-norm clip 1.0, Adam (wd 0.03 on weights, 0 on biases/norms) and a
per-step LR-schedule update. Synthetic ImageNet-shaped inputs (random [B,3,224,224], 1000 classes)
and random-init weights: there is no dataset or checkpoint access.

Prints ONE JSON line (rank 0). ``value`` is whole-job images/sec = global_batch * steps / max-rank
elapsed time, where the timed region is bracketed by barrier + device synchronize on both sides.

  python bench.py                          # 1 GPU, batch 256
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
  python bench.py --impl torch             # reference-style eager PyTorch (nn modules + autocast bf16)
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=None,
                   help="per-GPU batch (default: ViT-B/16 256 on 1 GPU, 512 per GPU on more; ViT-L/16 128; ViT-H/14 256)")
    p.add_argument("--model", default="vit_b16")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=1000)
    p.add_argument("--impl", choices=["fused", "torch"], default="fused")
    p.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16",
                   help="fp8: encoder forward GEMMs in e4m3 with delayed scaling (ViT-H/14 fp8 config)")
    p.add_argument("--fp8-bf16-dgrad", action="store_true", help="fp8 mode: keep the dgrad GEMMs bf16 (A/B)")
    p.add_argument("--fp8-bf16-wgrad", action="store_true",
                   help="fp8 mode: keep the weight-gradient GEMMs bf16 (fp8 weight gradients are the default)")
    p.add_argument("--fp8-grad", choices=["e5m2", "e4m3"], default="e4m3",
                   help="fp8 mode: the gradients' format in the dgrad / wgrad GEMMs (e4m3, the default since round 6: half "
                        "the gradient error of e5m2 at the same speed, profiles/r6/e4m3)")
    p.add_argument("--fp8-wgrad", action="store_true",
                   help="fp8 mode: fp8 weight gradients (the default since round 6; kept so older command lines parse)")
    p.add_argument("--profile-out", default=None, help="write a torch.profiler kernel table here")
    p.add_argument("--force-ddp", action="store_true", help="wrap in DDP even with one process (exercises the comm path)")
    p.add_argument("--pg-only", action="store_true", help="initialise a world-1 RCCL process group but do not wrap in DDP (A/B)")
    p.add_argument("--comm", choices=["auto", "torch"], default="auto", help="DDP gradient transport (torch.distributed / RCCL)")
    p.add_argument("--bucket-mb", type=float, default=28.0)
    p.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32",
                   help="gradient wire format of the DDP all-reduce (bf16: persistent bf16 mirror of the buckets)")
    p.add_argument("--metrics-jsonl", default=None,
                   help="per-step JSONL (step ms, img/s, lr, loss, grad-norm, per-bucket all-reduce ms) of the timed steps")
    p.add_argument("--graph", action="store_true", help="replay the whole training step as one captured hipGraph")
    p.add_argument("--infer", action="store_true",
                   help="serving throughput instead: eval-mode forward under inference_mode (no backward / optimizer)")
    p.add_argument("--serial-wgrad", action="store_true",
                   help="weight-gradient GEMMs on the main stream (no side stream): clean per-kernel times for profiles")
    p.add_argument("--side-window", type=int, default=None,
                   help="A/B: weight-gradient batches whose inputs stay held at once (0 = no count bound)")
    p.add_argument("--side-hold-gb", type=float, default=None,
                   help="A/B: GB of weight-gradient inputs held at once (0 = until the end of backward)")
    p.add_argument("--no-gemm-tail", action="store_true",
                   help="A/B: no split-K tail on the last dispatch round of the one-tile-per-workgroup GEMMs")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="process-group transport for --gpus > 1: nccl = RCCL (production); gloo = test-only, every rank "
                        "on the same GPU (LOCAL_RANK mod device count), to exercise this multi-rank path on a 1-GPU box")
    p.add_argument("--main-prio", type=int, default=-1,
                   help="run the step on a stream of this priority: -1 (default) puts the dgrad chain above the weight-gradient side stream; 0 = default stream")
    return p.parse_args()


MODEL_NAMES = {"vit_b16": "ViT-B/16", "vit_l16": "ViT-L/16", "vit_h14": "ViT-H/14"}

# Per-GPU batch when --batch is not given: BASELINE config 2 (ViT-B/16, 1 GPU) is batch 256; the
# data-parallel configs use a per-GPU batch sized to fit one MI355X's 288 GB with margin (configs 3-5:
# ViT-B/16 512 -> 4096 on 8 GPUs; ViT-L/16@384 128; ViT-H/14 fp8 256, ~134 GB measured at b256).
PER_GPU_BATCH = {"vit_b16": 512, "vit_l16": 128, "vit_h14": 256}
# Peak-memory model for the fail-fast check, fitted to measured peaks (bench.py's peak_mem_gb):
# GB = fixed + per_image * batch * (tokens / tokens_ref); profiles/r4/final2 and profiles/r5/configs
MEM_MODEL = {  # model: (fixed GB, GB per image at the reference token count, reference tokens)
    "vit_b16": (2.0, 0.0622, 197),    # b256: 17.9 GB
    "vit_l16": (5.5, 0.4556, 577),    # 384 px b128: 63.8 GB
    "vit_h14": (12.0, 0.477, 257),    # fp8 b256: 134.2 GB
}


def default_per_gpu_batch(model: str, world: int) -> int:
    if model == "vit_b16" and world == 1:
        return 256
    return PER_GPU_BATCH.get(model, 256 if world == 1 else 512)


def estimate_peak_gb(model: str, image_size: int, batch: int) -> float | None:
    """Peak device memory of one training step (None: model not calibrated)."""
    from pytorch_vit_paper_replication_amd.models.presets import PRESETS

    if model not in MEM_MODEL or model not in PRESETS:
        return None
    fixed, per_img, tok_ref = MEM_MODEL[model]
    tokens = (image_size // int(PRESETS[model]["patch_size"])) ** 2 + 1
    return fixed + per_img * batch * tokens / tok_ref


def describe(args, world: int) -> dict:
    """The run's configuration as reported (and as BASELINE.json names it), from the arguments and the
    world size alone: no GPU or model needed (tests/test_bench_cli.py checks configs 2-5 with it)."""
    from pytorch_vit_paper_replication_amd.models.presets import PRESETS

    per_gpu = args.batch or default_per_gpu_batch(args.model, world)
    name = MODEL_NAMES.get(args.model, args.model)
    patch = int(PRESETS[args.model]["patch_size"]) if args.model in PRESETS else 16
    if args.infer:
        metric = f"inference images/sec (whole node) {name} {args.image_size}px {args.dtype}"
    elif (name, args.image_size, args.dtype) == ("ViT-B/16", 224, "bf16"):
        metric = "images/sec (whole node) ViT-B/16 224px bf16 at 1/2/4/8 MI355X"
    else:
        metric = f"images/sec (whole node) {name} {args.image_size}px {args.dtype}"
    return {"name": name, "metric": metric, "per_gpu_batch": per_gpu, "global_batch": per_gpu * world,
            "seq_len": (args.image_size // patch) ** 2 + 1, "parallelism": f"dp{world}",
            "ddp": world > 1 or args.force_ddp}


def _relaunch_distributed(n: int) -> int:
    """``python bench.py --gpus N`` without a torchrun environment: run the same command under
    ``torch.distributed.run`` (one rank per GPU, rendezvous on 127.0.0.1) as a CHILD process and return
    its exit code. Nothing has touched the GPU yet in this process."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_relaunch_distributed(args.gpus))
    if args.impl == "torch":
        os.environ["PVR_DISABLE_FUSED"] = "1"
    import torch

    sys.path.insert(0, os.environ.get("PVR_PKG_ROOT") or os.path.dirname(os.path.abspath(__file__)))  # PVR_PKG_ROOT: an A/B build
    from pytorch_vit_paper_replication_amd.models import vit
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay
    from pytorch_vit_paper_replication_amd.ops.fused_vit import backward, cross_entropy
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel, barrier, init_distributed

    if args.serial_wgrad or args.side_window is not None or args.side_hold_gb is not None:
        from pytorch_vit_paper_replication_amd.runtime import param_store

        if args.serial_wgrad:
            param_store.SIDE_WGRAD = False
        if args.side_window is not None:
            param_store.SIDE_WINDOW = args.side_window
        if args.side_hold_gb is not None:
            param_store.SIDE_HOLD_BYTES = int(args.side_hold_gb * 2**30)
    if args.backend == "gloo":  # test transport: ranks share the GPU(s); gradients travel over gloo
        rank, world, _ = init_distributed(backend="gloo")
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        torch.cuda.set_device(device)
    else:
        rank, world, device = init_distributed()
    if args.no_gemm_tail and args.impl == "fused":
        from pytorch_vit_paper_replication_amd import _ext

        _ext.ext().set_gemm_tail(False)
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU (torch.distributed.run)")
    if (args.force_ddp or args.pg_only) and not torch.distributed.is_initialized():
        import datetime

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=device,
                                             timeout=datetime.timedelta(seconds=600))
    desc = describe(args, world)
    per_gpu = desc["per_gpu_batch"]
    est = estimate_peak_gb(args.model, args.image_size, per_gpu) if not args.infer else None
    hbm = torch.cuda.get_device_properties(device).total_memory / 2**30
    if est is not None and est > 0.95 * hbm:
        raise SystemExit(f"bench.py: {desc['name']} at {args.image_size} px needs ~{est:.0f} GB per GPU at batch {per_gpu} "
                         f"(device has {hbm:.0f} GB); pass a smaller --batch (default {default_per_gpu_batch(args.model, world)})")
    torch.manual_seed(1234)

    model = vit(args.model, image_size=args.image_size, num_classes=args.num_classes).to(device)
    if args.dtype == "fp8":
        model.enable_fp8(dgrad=not args.fp8_bf16_dgrad, wgrad=not args.fp8_bf16_wgrad and not args.fp8_bf16_dgrad,
                         grad_fmt=args.fp8_grad)
    groups = param_groups_weight_decay(model, 0.03)
    total_steps = args.warmup + args.steps
    if args.impl == "fused":
        opt = FusedAdam(groups, lr=1e-3, betas=(0.9, 0.999))
    else:
        opt = torch.optim.Adam(groups, lr=1e-3, betas=(0.9, 0.999))
    sched = warmup_linear_decay(opt, max(total_steps, 20), 0.05)
    use_ddp = desc["ddp"]
    net = DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb, comm=args.comm,
                                  comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else None,
                                  timing=bool(args.metrics_jsonl)) if use_ddp else model

    g = torch.Generator(device=device).manual_seed(rank)
    x = torch.rand(per_gpu, 3, args.image_size, args.image_size, device=device, generator=g)
    y = torch.randint(0, args.num_classes, (per_gpu,), device=device, generator=g)

    def infer_step():
        amp = torch.autocast("cuda", dtype=torch.bfloat16) if args.impl == "torch" else contextlib.nullcontext()
        with torch.inference_mode(), amp:
            return model(x).float().logsumexp(-1).mean()

    def step():
        net.train()
        if args.impl == "fused":
            logits = net(x)
            loss = cross_entropy(logits, y)
            opt.zero_grad()
            backward(loss)
            opt.step(clip_norm=1.0)
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = net(x)
                loss = torch.nn.functional.cross_entropy(logits.float(), y)
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
            opt.step()
        sched.step()
        return loss

    if args.infer:
        model.eval()
        step = infer_step  # noqa: F811
        if args.graph:
            # serving at small batch: the eval forward captured once as a hipGraph, replayed per batch
            if args.impl != "fused":
                raise SystemExit("--infer --graph: fused path only")
            side = torch.cuda.Stream(device=device)
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side):
                for _ in range(3):
                    infer_step()
            torch.cuda.current_stream(device).wait_stream(side)
            torch.cuda.synchronize()
            ig = torch.cuda.CUDAGraph()
            with torch.cuda.graph(ig):
                static_out = infer_step()

            def step():  # noqa: F811
                ig.replay()
                return static_out
            args.warmup = max(args.warmup, 1)
    if args.graph and not args.infer:
        if args.impl != "fused" or use_ddp:
            raise SystemExit("--graph: single-process fused path only")
        from pytorch_vit_paper_replication_amd.runtime.graph import GraphedTrainStep

        graphed = GraphedTrainStep(model, opt, cross_entropy, x, y, clip_norm=1.0, warmup=max(1, args.warmup),
                                   scheduler=sched)
        step = graphed  # noqa: F811  (each call: graph_prepare + hipGraphLaunch + LR schedule step)
        args.warmup = 0
    stream_ctx = contextlib.nullcontext()
    if args.main_prio != 0:
        main_stream = torch.cuda.Stream(device=device, priority=args.main_prio)
        main_stream.wait_stream(torch.cuda.current_stream(device))
        stream_ctx = torch.cuda.stream(main_stream)
    with stream_ctx:
        for _ in range(args.warmup):
            loss = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    logger = None
    if args.metrics_jsonl:
        from pytorch_vit_paper_replication_amd.utils.metrics import StepLogger

        # resolved after the timed region (no flush, hence no host sync, inside it)
        logger = StepLogger(args.metrics_jsonl, flush_every=args.steps + 1, rank=rank, world=world, device=device)
    t0 = time.perf_counter()
    with stream_ctx:
        for _ in range(args.steps):
            if logger is None:
                loss = step()
                continue
            lr = opt.param_groups[0]["lr"]
            logger.begin()
            loss = step()
            logger.end(batch=per_gpu, loss=loss, grad_norm=getattr(opt, "last_grad_norm", None), lr=lr,
                       ddp=net if use_ddp else None)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if use_ddp:  # the slowest rank's time (CPU tensor on the gloo test transport)
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if args.backend == "nccl" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())
    if logger is not None:
        logger.close()

    if args.profile_out and rank == 0:
        from pytorch_vit_paper_replication_amd.utils.profiling import profile_steps

        profile_steps(step, steps=2, out_path=args.profile_out)

    global_batch = desc["global_batch"]
    ips = global_batch * args.steps / elapsed
    name = desc["name"]
    seq = desc["seq_len"]
    if rank == 0:
        out = {
            "metric": desc["metric"],
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "bf16" else (
                "fp8 (e4m3 forward GEMMs; bf16 backward/attention/norms)" if args.fp8_bf16_dgrad else
                f"fp8 (e4m3 forward GEMMs, {args.fp8_grad}-gradient dgrad and wgrad GEMMs; bf16 attention/norms)"
                if not args.fp8_bf16_wgrad else
                f"fp8 (e4m3 forward GEMMs, {args.fp8_grad}-gradient dgrad GEMMs; bf16 wgrad/attention/norms)"),
            "data": f"synthetic (random [B,3,{args.image_size},{args.image_size}] in [0,1), {args.num_classes} classes, "
                    "random-init weights)",
            "config": {"model": name, "global_batch": global_batch, "per_gpu_batch": per_gpu, "seq_len": seq,
                       "image_size": args.image_size, "parallelism": desc["parallelism"], "impl": args.impl + ("+hipgraph" if args.graph else ""),
                       "grad_transport": (net.transport + f" {args.comm_dtype} wire" + (" (gloo test transport, shared GPU)"
                                          if args.backend == "gloo" else "")) if use_ddp else "none",
                       "optimizer": "none (inference: eval forward under inference_mode)" if args.infer else
                       "Adam(wd=0.03 decay group) + clip 1.0 + warmup/linear-decay LR",
                       "dropout": "off (eval)" if args.infer else "0.1 (mlp, embedding)",
                       "final_loss": round(final_loss, 4),
                       # BASELINE configs 2 / 3: 256 images on one GPU, 512 per GPU on 2-8 (global 4096 at 8);
                       # efficiency against 1 GPU at 512 (bench.py --batch 512 --force-ddp) keeps per-GPU work fixed
                       "scaling_note": "per-GPU batch 256 at 1 GPU (config 2), 512 at 2-8 GPUs (config 3)"
                       if name == "ViT-B/16" and args.batch is None and not args.infer else None,
                       "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 2)},
        }
        print(json.dumps(out), flush=True)
    if use_ddp:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
