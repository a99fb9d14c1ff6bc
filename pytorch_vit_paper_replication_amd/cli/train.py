"""Command-line trainer (replaces the reference's broken GM/train.py).

Examples::

    python -m pytorch_vit_paper_replication_amd.cli.train --model vit_b16 --synthetic --epochs 2 --batch-size 64
    python -m pytorch_vit_paper_replication_amd.cli.train --model tinyvgg --train-dir data/pizza_steak_sushi/train \
        --test-dir data/pizza_steak_sushi/test --image-size 64
    torchrun --nproc-per-node 8 -m pytorch_vit_paper_replication_amd.cli.train --synthetic ...   # RCCL DP
    python -m pytorch_vit_paper_replication_amd.cli.train --model vit_h14 --synthetic --dtype fp8   # BASELINE config 5
"""
from __future__ import annotations

import argparse
import contextlib

import torch


def _is_rank0() -> bool:
    d = torch.distributed
    return not (d.is_available() and d.is_initialized()) or d.get_rank() == 0


def build_parser():
    p = argparse.ArgumentParser(description="Train a ViT (or TinyVGG) with the MI355X-native engine")
    p.add_argument("--model", default="vit_b16", help="vit_b16 | vit_l16 | vit_h14 | vit_tiny_test | tinyvgg")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=None)
    p.add_argument("--train-dir", default=None)
    p.add_argument("--test-dir", default=None)
    p.add_argument("--synthetic", action="store_true", help="synthetic ImageNet-shaped data")
    p.add_argument("--synthetic-train-len", type=int, default=512)
    p.add_argument("--synthetic-test-len", type=int, default=128)
    p.add_argument("--epochs", type=int, default=5, help="total epochs (a --resume run trains the rest)")
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--weight-decay", type=float, default=0.03)
    p.add_argument("--warmup-frac", type=float, default=0.05)
    p.add_argument("--max-grad-norm", type=float, default=1.0)
    p.add_argument("--num-workers", type=int, default=4)
    p.add_argument("--hidden-units", type=int, default=10)
    p.add_argument("--save-dir", default="models")
    p.add_argument("--save-name", default=None)
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--resume", default=None)
    p.add_argument("--metrics", default=None, help="append per-epoch JSONL metrics here")
    p.add_argument("--torch-optimizer", action="store_true", help="use torch.optim.Adam instead of FusedAdam")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16",
                   help="fp8: the encoder GEMMs in fp8 with delayed scaling (ViT.enable_fp8; GPU fused path only)")
    p.add_argument("--fp8-grad", choices=["e4m3", "e5m2"], default="e4m3", help="fp8: the gradients' format")
    p.add_argument("--fp8-bf16-wgrad", action="store_true", help="fp8: keep the weight-gradient GEMMs bf16")
    p.add_argument("--dropout", type=float, default=None,
                   help="override the MLP and embedding dropout of the ViT preset (0.1 = the reference's)")
    p.add_argument("--deterministic", action="store_true",
                   help="fixed-order reductions instead of float atomics: bitwise-repeatable gradients")
    p.add_argument("--bucket-mb", type=float, default=28.0, help="DDP gradient bucket size (MiB)")
    p.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32", help="DDP all-reduce wire format")
    return p


def main(argv=None) -> int:
    from .. import engine
    from ..data import create_dataloaders, create_synthetic_dataloaders
    from ..data.transforms import default_vit_transform
    from ..models import TinyVGG, vit
    from ..optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay
    from ..parallel import DistributedDataParallel, init_distributed, is_dist
    from .. import _ext
    from ..utils import load_checkpoint, save_model, set_seeds

    args = build_parser().parse_args(argv)
    if args.dtype == "fp8" and args.model == "tinyvgg":
        raise SystemExit("--dtype fp8 applies to the ViT models")
    rank, world, device = init_distributed()
    set_seeds(args.seed)
    if args.synthetic or not args.train_dir:
        ncls = args.num_classes or 1000
        train_dl, test_dl, class_names = create_synthetic_dataloaders(
            args.batch_size, args.synthetic_train_len, args.synthetic_test_len, args.image_size, ncls,
            num_workers=0)
    else:
        tf = default_vit_transform(args.image_size)
        train_dl, test_dl, class_names = create_dataloaders(args.train_dir, args.test_dir, tf, args.batch_size,
                                                            num_workers=args.num_workers)
    ncls = args.num_classes or len(class_names)
    if args.model == "tinyvgg":
        model = TinyVGG(input_shape=3, hidden_units=args.hidden_units, output_shape=ncls)
    else:
        drop = {} if args.dropout is None else dict(mlp_dropout=args.dropout, embedding_dropout=args.dropout)
        model = vit(args.model, image_size=args.image_size, num_classes=ncls, **drop)
        if args.dtype == "fp8":  # before a resume: the checkpoint's fp8 scaling state needs it
            model.enable_fp8(wgrad=not args.fp8_bf16_wgrad, grad_fmt=args.fp8_grad)
    model.to(device)
    groups = param_groups_weight_decay(model, args.weight_decay)
    if args.torch_optimizer:
        opt = torch.optim.Adam(groups, lr=args.lr, betas=(0.9, 0.999))
    else:
        opt = FusedAdam(groups, lr=args.lr, betas=(0.9, 0.999))
    sched = warmup_linear_decay(opt, args.epochs * len(train_dl), args.warmup_frac)
    start_epoch, results = 0, None
    if args.resume:
        # --epochs is the TOTAL epoch count: a resumed run trains only the epochs not yet done, on the
        # same (restored) LR schedule, so it ends where the uninterrupted run would have
        info = load_checkpoint(args.resume, model, opt, sched)
        start_epoch, results = int(info["epoch"]), info["results"]
        if _is_rank0():
            print(f"[INFO] Resumed {args.resume} at epoch {start_epoch} of {args.epochs}")
    net = (DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb,
                                   comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else None)
           if is_dist() else model)
    with _ext.deterministic_mode() if args.deterministic else contextlib.nullcontext():
        engine.train(model=net, train_dataloader=train_dl, test_dataloader=test_dl, optimizer=opt,
                     loss_fn=torch.nn.CrossEntropyLoss(), lr_scheduler=sched, epochs=args.epochs, device=device,
                     max_grad_norm=args.max_grad_norm, checkpoint_dir=args.checkpoint_dir, metrics_path=args.metrics,
                     start_epoch=start_epoch, results=results)
    save_model(model, args.save_dir, args.save_name or f"{args.model}_{args.epochs}_epochs.pth")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
