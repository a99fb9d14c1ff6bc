"""Training-trajectory parity at full model size: the fused HIP path (bf16 MFMA kernels, FusedAdam)
vs the reference-style PyTorch fp32 path (nn modules, torch.optim.Adam, clip_grad_norm_) and the same
PyTorch path under autocast bf16 (separates bf16 rounding from kernel behaviour), same init,
same batches, same recipe (reference MAIN.ipynb:2818-2824 Adam + L2 wd 0.03 on the decay group,
GM/engine.py:63 clip 1.0, MAIN.ipynb:2896-2912 5 % linear warmup then linear decay per batch).

Data: a learnable synthetic task (no dataset download here): each class has a fixed random template,
one colour per 16x16 patch (a random [3, 14, 14] grid upsampled to 224 px); a sample is
0.7 * template + 0.3 * uniform noise. Train and held-out sets are drawn once.
Dropout defaults to 0 so the two trajectories are comparable step by step (dropout RNG streams differ
between the paths by construction).

usage (GPU): python scripts/convergence_check.py [--model vit_b16] [--steps 300] [--batch 64] [--lr 1e-4]
Prints the per-step losses every --log steps and ONE JSON summary line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def make_data(n, classes, image, gen, device, templates):
    y = torch.randint(0, classes, (n,), generator=gen, device=device)
    noise = torch.rand(n, 3, image, image, generator=gen, device=device)
    return 0.7 * templates[y] + 0.3 * noise, y


def run(path, args, init_sd, data):
    from pytorch_vit_paper_replication_amd.models import vit
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay

    fused = path.startswith("fused")
    os.environ["PVR_DISABLE_FUSED"] = "0" if fused else "1"
    amp = torch.autocast("cuda", dtype=torch.bfloat16, enabled=path == "reference_bf16")
    dev = torch.device("cuda")
    model = vit(args.model, image_size=args.image_size, num_classes=args.classes,
                mlp_dropout=args.dropout, embedding_dropout=args.dropout).to(dev)
    model.load_state_dict(init_sd)
    # the gradient format is explicit: the fp8 default changed to e4m3 in late round 6, and the arms keep
    # their meaning (the e4m3-study runs of seeds 6-11 predate this: their "fused_fp8w" arm ran e4m3)
    if path == "fused_fp8":
        model.enable_fp8(wgrad=False, grad_fmt="e5m2")  # e4m3 forward, e5m2-gradient dgrad GEMMs (wgrad bf16)
    elif path == "fused_fp8w":
        model.enable_fp8(dgrad=True, wgrad=True, grad_fmt="e5m2")  # + e5m2 x e4m3 weight-gradient GEMMs
    elif path == "fused_fp8w4":
        model.enable_fp8(dgrad=True, wgrad=True, grad_fmt="e4m3")  # the same with e4m3 gradients
    groups = param_groups_weight_decay(model, 0.03)
    opt = FusedAdam(groups, lr=args.lr) if fused else torch.optim.Adam(groups, lr=args.lr)
    sched = warmup_linear_decay(opt, args.steps, 0.05)
    (xtr, ytr), (xte, yte) = data
    losses = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # --stop-at: train only the first steps of the --steps schedule (mid-training comparisons)
    for s in range(min(args.steps, getattr(args, "stop_at", 0) or args.steps)):
        lo = (s * args.batch) % xtr.shape[0]
        x, y = xtr[lo:lo + args.batch], ytr[lo:lo + args.batch]
        model.train()
        if fused:
            loss = cross_entropy(model(x), y)
            opt.zero_grad()
            loss.backward()
            opt.step(clip_norm=1.0)
        else:
            with amp:
                logits = model(x)
            loss = F.cross_entropy(logits.float(), y)
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
            opt.step()
        sched.step()
        losses.append(float(loss.item()))
        if (s + 1) % args.log == 0:
            print(f"[{path}] step {s + 1:4d} loss {losses[-1]:.4f}", flush=True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    model.eval()
    correct, tot_loss = 0, 0.0
    with torch.inference_mode(), amp:
        for lo in range(0, xte.shape[0], args.batch):
            logits = model(xte[lo:lo + args.batch]).float()
            tot_loss += float(F.cross_entropy(logits, yte[lo:lo + args.batch], reduction="sum"))
            correct += int((logits.argmax(-1) == yte[lo:lo + args.batch]).sum())
    os.environ["PVR_DISABLE_FUSED"] = "0"
    return {"losses": losses, "test_loss": tot_loss / xte.shape[0], "test_acc": correct / xte.shape[0],
            "train_s": round(elapsed, 2)}


def _with_reference(args, init_sd, data, fused, k):
    ref = run("reference", args, init_sd, data)
    ref16 = run("reference_bf16", args, init_sd, data)
    lf, lr_ = fused["losses"], ref["losses"]
    return {
        "model": args.model, "steps": args.steps, "batch": args.batch, "lr": args.lr, "dropout": args.dropout,
        "fused": {"first": lf[0], "last10pct_mean": sum(lf[-k:]) / k, "test_loss": fused["test_loss"],
                  "test_acc": fused["test_acc"], "train_s": fused["train_s"]},
        "reference_fp32": {"first": lr_[0], "last10pct_mean": sum(lr_[-k:]) / k, "test_loss": ref["test_loss"],
                           "test_acc": ref["test_acc"], "train_s": ref["train_s"]},
        "reference_autocast_bf16": {"first": ref16["losses"][0], "last10pct_mean": sum(ref16["losses"][-k:]) / k,
                                    "test_loss": ref16["test_loss"], "test_acc": ref16["test_acc"],
                                    "train_s": ref16["train_s"]},
        "max_abs_loss_diff_first10": max(abs(a - b) for a, b in zip(lf[:10], lr_[:10])),
        "mean_abs_loss_diff": sum(abs(a - b) for a, b in zip(lf, lr_)) / len(lf),
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="vit_b16")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--classes", type=int, default=10)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--train-size", type=int, default=2048)
    p.add_argument("--test-size", type=int, default=512)
    p.add_argument("--log", type=int, default=10)
    p.add_argument("--fp8", action="store_true", help="also train the fused path with enable_fp8() (fp8 GEMMs)")
    p.add_argument("--no-reference", action="store_true",
                   help="skip the two PyTorch paths (large models: fused bf16 vs fused fp8 only)")
    p.add_argument("--fp8-study", type=int, default=0, metavar="SEEDS",
                   help="seed study: SEEDS inits x {fused bf16, fp8 fwd+dgrad, fp8 fwd+dgrad+wgrad}; prints the "
                        "per-variant mean / spread of the final loss and held-out accuracy")
    p.add_argument("--variants", default="fused,fused_fp8,fused_fp8w",
                   help="seed study: paths to train per seed (fused = bf16; fused_fp8 = fp8 fwd+dgrad; fused_fp8w = "
                        "+ fp8 weight gradients; fused_fp8w4 = the same with e4m3 gradients)")
    p.add_argument("--seed-start", type=int, default=0, help="seed study: first seed (studies split over runs)")
    p.add_argument("--stop-at", type=int, default=0, help="train only this many steps of the --steps schedule")
    p.add_argument("--checkpoints", default="", help="seed study: comma-separated steps whose windowed mean loss "
                   "(the --window steps ending there) is recorded per run (JSON line '[ckpt] ...')")
    p.add_argument("--window", type=int, default=20)
    args = p.parse_args()
    if args.fp8_study:
        return fp8_study(args)

    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import vit

    assert torch.cuda.is_available(), "GPU script"
    _ext.ext()  # the fused path must be the HIP extension, not a fallback
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(0)
    g = args.image_size // 16
    templates = torch.rand(args.classes, 3, g, g, generator=gen, device=dev)
    templates = F.interpolate(templates, size=(args.image_size, args.image_size), mode="nearest")
    data = (make_data(args.train_size, args.classes, args.image_size, gen, dev, templates),
            make_data(args.test_size, args.classes, args.image_size, gen, dev, templates))
    torch.manual_seed(0)
    init_sd = {k: v.clone() for k, v in vit(args.model, image_size=args.image_size, num_classes=args.classes,
                                          mlp_dropout=args.dropout, embedding_dropout=args.dropout).state_dict().items()}
    fused = run("fused", args, init_sd, data)
    lf = fused["losses"]
    k = max(1, args.steps // 10)
    if args.no_reference:
        summary = {"model": args.model, "steps": args.steps, "batch": args.batch, "lr": args.lr, "dropout": args.dropout,
                   "fused": {"first": lf[0], "last10pct_mean": sum(lf[-k:]) / k, "test_loss": fused["test_loss"],
                             "test_acc": fused["test_acc"], "train_s": fused["train_s"]}}
    else:
        summary = _with_reference(args, init_sd, data, fused, k)
    if args.fp8:
        f8 = run("fused_fp8", args, init_sd, data)
        summary["fused_fp8"] = {"first": f8["losses"][0], "last10pct_mean": sum(f8["losses"][-k:]) / k,
                                "test_loss": f8["test_loss"], "test_acc": f8["test_acc"], "train_s": f8["train_s"],
                                "max_abs_loss_diff_vs_fused_first50": max(abs(a - b) for a, b in zip(f8["losses"][:50], lf[:50]))}
    print(json.dumps(summary), flush=True)


def fp8_study(args):
    """Learning-phase parity of the fp8 paths: for each seed, the same init and batch order through the
    fused bf16 path, fp8 forward + dgrad (ViT.enable_fp8 default) and fp8 forward + dgrad + wgrad; the
    question is whether each fp8 variant's final loss / held-out accuracy falls inside the bf16 seed
    spread."""
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import vit

    assert torch.cuda.is_available(), "GPU script"
    _ext.ext()
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(0)
    g = args.image_size // 16
    templates = F.interpolate(torch.rand(args.classes, 3, g, g, generator=gen, device=dev),
                              size=(args.image_size, args.image_size), mode="nearest")
    tr = make_data(args.train_size, args.classes, args.image_size, gen, dev, templates)
    te = make_data(args.test_size, args.classes, args.image_size, gen, dev, templates)
    k = max(1, args.steps // 10)
    res = {v: [] for v in args.variants.split(",")}
    ckpts = [int(c) for c in args.checkpoints.split(",") if c]
    for seed in range(args.seed_start, args.seed_start + args.fp8_study):
        torch.manual_seed(seed)
        init_sd = {n: t.clone() for n, t in vit(args.model, image_size=args.image_size, num_classes=args.classes,
                                               mlp_dropout=args.dropout, embedding_dropout=args.dropout).state_dict().items()}
        perm = torch.randperm(tr[0].shape[0], generator=torch.Generator().manual_seed(seed)).to(dev)
        data = ((tr[0][perm], tr[1][perm]), te)
        for v in res:
            r = run(v, args, init_sd, data)
            res[v].append({"final_loss": sum(r["losses"][-k:]) / k, "test_acc": r["test_acc"], "test_loss": r["test_loss"]})
            if ckpts:  # windowed mean loss ending at each checkpoint step (1-based)
                w = {c: sum(r["losses"][c - args.window:c]) / args.window for c in ckpts if c <= len(r["losses"])}
                print("[ckpt] " + json.dumps({"seed": seed, "variant": v, "window": args.window, "loss": w,
                                              "train_s": r["train_s"]}), flush=True)
            print(f"[study] seed {seed} {v}: final loss {res[v][-1]['final_loss']:.4f} test acc {r['test_acc']:.3f} "
                  f"test loss {r['test_loss']:.4f}", flush=True)

    def stats(xs):
        m = sum(xs) / len(xs)
        return {"mean": round(m, 4), "min": round(min(xs), 4), "max": round(max(xs), 4),
                "std": round((sum((x - m) ** 2 for x in xs) / max(1, len(xs) - 1)) ** 0.5, 4)}

    summary = {"model": args.model, "steps": args.steps, "batch": args.batch, "lr": args.lr, "seeds": args.fp8_study}
    for v, rs in res.items():
        summary[v] = {key: stats([r[key] for r in rs]) for key in ("final_loss", "test_acc", "test_loss")}
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
