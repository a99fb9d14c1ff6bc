"""End-to-end GPU tests of the fused training path.

* the reference engine (going_modular.engine.train) drives the fused HIP ViT on cuda:0 and the loss
  falls on a fixed synthetic batch (dropout on, the real recipe: Adam + clip + warmup/decay),
* several fused optimizer steps track a PyTorch fp32 training run of the same model,
* DDP over RCCL with world_size=1 (the only RCCL topology a 1-GPU box offers) produces exactly the
  non-DDP gradients, and the engine runs under it.
"""
import os
import socket

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CFG = dict(image_size=64, patch_size=16, num_transformer_layer=2, num_heads=2, embedding_dim=128, mlp_size=256,
           num_classes=10)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_engine_trains_fused_vit_on_gpu(capsys):
    from going_modular import engine
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay

    assert _ext.available()
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    model = ViT(**CFG)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(32, 3, 64, 64, generator=g)
    y = torch.randint(0, 10, (32,), generator=g)
    ds = torch.utils.data.TensorDataset(x, y)
    dl = torch.utils.data.DataLoader(ds, batch_size=16, shuffle=False)
    opt = FusedAdam(param_groups_weight_decay(model, 0.0), lr=2e-3)
    sched = warmup_linear_decay(opt, 6 * len(dl), 0.05)
    res = engine.train(model, dl, dl, opt, torch.nn.CrossEntropyLoss(), sched, epochs=6, device=dev)
    assert getattr(model, "_pvr_store", None) is not None, "fused path did not run"
    assert len(res["train_loss"]) == 6
    assert res["train_loss"][-1] < res["train_loss"][0]
    assert res["test_loss"][-1] < res["test_loss"][0]
    assert "Epoch: 6 | train_loss:" in capsys.readouterr().out


def test_fused_training_tracks_fp32_reference():
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay

    torch.manual_seed(0)
    cfg = dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)
    mf, mr = ViT(**cfg).cuda(), ViT(**cfg).cuda()
    mr.load_state_dict(mf.state_dict())
    of = FusedAdam(param_groups_weight_decay(mf, 0.03), lr=1e-3)
    orf = torch.optim.Adam(param_groups_weight_decay(mr, 0.03), lr=1e-3)
    x = torch.rand(8, 3, 64, 64, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    p0 = torch.cat([p.detach().reshape(-1).clone() for p in mf.parameters()])
    lf_hist, lr_hist = [], []
    for _ in range(5):
        loss = cross_entropy(mf(x), y)
        of.zero_grad()
        loss.backward()
        of.step(clip_norm=1.0)
        lf_hist.append(loss.item())
        os.environ["PVR_DISABLE_FUSED"] = "1"
        try:
            lr_ = F.cross_entropy(mr(x), y)
        finally:
            os.environ["PVR_DISABLE_FUSED"] = "0"
        orf.zero_grad()
        lr_.backward()
        torch.nn.utils.clip_grad_norm_(mr.parameters(), 1.0)
        orf.step()
        lr_hist.append(lr_.item())
    assert lf_hist[-1] < lf_hist[0]
    for a, b in zip(lf_hist, lr_hist):
        assert abs(a - b) < 3e-2 * max(1.0, abs(b)), (lf_hist, lr_hist)
    # Adam updates are ~sign(g) for tiny gradients, so compare the overall update direction
    uf = torch.cat([p.detach().reshape(-1) for p in mf.parameters()]) - p0
    ur = torch.cat([p.detach().reshape(-1) for p in mr.parameters()]) - p0
    cos = F.cosine_similarity(uf, ur, dim=0).item()
    assert cos > 0.9, f"fused vs fp32 update direction cosine {cos:.3f}"


def test_full_size_vit_b16_steps_track_fp32_reference():
    """ViT-B/16 at 224 px (the headline model): 8 training steps of the fused path against the
    PyTorch fp32 path from the same init on the same batches. scripts/convergence_check.py measured
    the two losses within 0.005 of each other for the first ~190 steps (profiles/conv/convergence_b16.md)."""
    from pytorch_vit_paper_replication_amd.models import vit
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay

    torch.manual_seed(0)
    kw = dict(num_classes=10, mlp_dropout=0.0, embedding_dropout=0.0)
    mf, mr = vit("vit_b16", **kw).cuda(), vit("vit_b16", **kw).cuda()
    mr.load_state_dict(mf.state_dict())
    of = FusedAdam(param_groups_weight_decay(mf, 0.03), lr=1e-4)
    orf = torch.optim.Adam(param_groups_weight_decay(mr, 0.03), lr=1e-4)
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = torch.rand(8, 16, 3, 224, 224, device="cuda", generator=g)
    ys = torch.randint(0, 10, (8, 16), device="cuda", generator=g)
    lf, lr_ = [], []
    for x, y in zip(xs, ys):
        loss = cross_entropy(mf(x), y)
        of.zero_grad()
        loss.backward()
        of.step(clip_norm=1.0)
        lf.append(loss.item())
        os.environ["PVR_DISABLE_FUSED"] = "1"
        try:
            l2 = F.cross_entropy(mr(x), y)
        finally:
            os.environ["PVR_DISABLE_FUSED"] = "0"
        orf.zero_grad()
        l2.backward()
        torch.nn.utils.clip_grad_norm_(mr.parameters(), 1.0)
        orf.step()
        lr_.append(l2.item())
    diffs = [abs(a - b) for a, b in zip(lf, lr_)]
    print(f"fused {lf}\nfp32  {lr_}\nmax |dloss| {max(diffs):.5f}")
    assert max(diffs) < 2e-2, (lf, lr_)


def test_ddp_rccl_world1_matches_local():
    import torch.distributed as dist

    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        torch.manual_seed(0)
        cfg = dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)
        m1, m2 = ViT(**cfg).to(dev), ViT(**cfg).to(dev)
        m2.load_state_dict(m1.state_dict())
        ddp = DistributedDataParallel(m1, bucket_cap_mb=0.25)
        x = torch.rand(4, 3, 64, 64, device=dev)
        y = torch.randint(0, 10, (4,), device=dev)
        for _ in range(2):
            for m in (m1, m2):
                for p in m.parameters():
                    if p.grad is not None:
                        p.grad.zero_()
            cross_entropy(ddp(x), y).backward()
            cross_entropy(m2(x), y).backward()
        torch.cuda.synchronize()
        assert len(ddp._buckets) > 1
        assert ddp.transport == "torch-nccl"
        for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
            assert torch.allclose(p1.grad, p2.grad, rtol=1e-4, atol=1e-5), n
    finally:
        dist.destroy_process_group()


def test_ddp_callbacks_run_on_the_callers_stream():
    """bench.py trains on a high-priority, non-default stream: the end-of-backward callbacks that join
    the side stream and the gradient all-reduces (DDP) must then order that stream, not the default one."""
    import torch.distributed as dist

    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        torch.manual_seed(0)
        m = ViT(**CFG).to(dev)
        ddp = DistributedDataParallel(m, bucket_cap_mb=0.25)
        x = torch.rand(4, 3, 64, 64, device=dev)
        y = torch.randint(0, 10, (4,), device=dev)
        seen = []
        fin = ddp._finalize

        def spy():
            seen.append(torch.cuda.current_stream(dev).stream_id)
            fin()

        ddp._finalize = spy
        s = torch.cuda.Stream(device=dev, priority=-1)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        assert ddp.transport == "torch-nccl"
        assert seen and all(v == s.stream_id for v in seen), (seen, s.stream_id)
    finally:
        dist.destroy_process_group()


def test_feature_extractor_fused_gpu():
    """Frozen backbone + new head on the fused path: only the head moves (MAIN.ipynb:4111-4130)."""
    from pytorch_vit_paper_replication_amd.models import ViT, feature_extractor
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam

    torch.manual_seed(0)
    m = feature_extractor(ViT(**CFG), num_classes=3, seed=0).cuda()
    frozen = {n: p.detach().clone() for n, p in m.named_parameters() if not p.requires_grad}
    head0 = m.classifier[0].weight.detach().clone()
    opt = FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    x = torch.rand(8, 3, 64, 64, device="cuda")
    y = torch.randint(0, 3, (8,), device="cuda")
    for _ in range(3):
        loss = cross_entropy(m(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step(clip_norm=1.0)
    torch.cuda.synchronize()
    assert getattr(m, "_pvr_store", None) is not None
    assert not torch.equal(m.classifier[0].weight, head0)
    for n, p in m.named_parameters():
        if n in frozen:
            assert torch.equal(p, frozen[n]), n


def test_graphed_train_step_matches_eager():
    """hipGraph replay of the full fused step (fwd, bwd, clip, Adam, LR schedule) tracks eager."""
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay
    from pytorch_vit_paper_replication_amd.runtime.graph import GraphedTrainStep

    torch.manual_seed(0)
    cfg = dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)
    ma, mb = ViT(**cfg).cuda(), ViT(**cfg).cuda()
    mb.load_state_dict(ma.state_dict())
    oa = FusedAdam(param_groups_weight_decay(ma, 0.03), lr=1e-3)
    ob = FusedAdam(param_groups_weight_decay(mb, 0.03), lr=1e-3)
    sa, sb = warmup_linear_decay(oa, 20, 0.1), warmup_linear_decay(ob, 20, 0.1)
    x = torch.rand(8, 3, 64, 64, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    la = []
    for _ in range(3 + 4):
        ma.train()
        loss = cross_entropy(ma(x), y)
        oa.zero_grad()
        loss.backward()
        oa.step(clip_norm=1.0)
        sa.step()
        la.append(loss.item())
    g = GraphedTrainStep(mb, ob, cross_entropy, x, y, clip_norm=1.0, warmup=3, scheduler=sb)
    lb = [g().item() for _ in range(4)]
    torch.cuda.synchronize()
    assert ob.step_count == oa.step_count == 7
    for a, b in zip(la[3:], lb):
        assert abs(a - b) < 2e-2 * max(1.0, abs(a)), (la, lb)
    for (n, p1), p2 in zip(ma.named_parameters(), mb.parameters()):
        assert torch.allclose(p1, p2, rtol=2e-2, atol=2e-4), n


def test_nonfinite_gradient_skips_step():
    """Failure detection: an inf/nan gradient is caught by the fused norm kernel and the Adam step is
    skipped on the device (no host sync), leaving parameters and moments untouched."""
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam

    torch.manual_seed(0)
    m = ViT(**dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)).cuda()
    opt = FusedAdam(m.parameters(), lr=1e-2)
    x = torch.rand(4, 3, 64, 64, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")
    loss = cross_entropy(m(x), y)
    opt.zero_grad()
    loss.backward()
    before = [p.detach().clone() for p in m.parameters()]
    m.classifier[0].weight.grad[0, 0] = float("inf")
    opt.step(clip_norm=1.0)
    torch.cuda.synchronize()
    assert not torch.isfinite(opt.last_grad_norm).item()
    for p0, p in zip(before, m.parameters()):
        assert torch.equal(p0, p)
    # the next finite step proceeds normally
    loss = cross_entropy(m(x), y)
    opt.zero_grad()
    loss.backward()
    opt.step(clip_norm=1.0)
    torch.cuda.synchronize()
    assert any(not torch.equal(p0, p) for p0, p in zip(before, m.parameters()))


def test_side_stream_matches_serial_weight_gradients(monkeypatch):
    """Stream-ordering check for the weight-gradient side stream (SURVEY.md §5 race detection): three
    training steps with concurrent wgrads equal the serial ones (up to f32 atomic ordering)."""
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam

    from pytorch_vit_paper_replication_amd.runtime import param_store

    def run(side: bool):
        monkeypatch.setattr(param_store, "SIDE_WGRAD", side)
        torch.manual_seed(0)
        m = ViT(**dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)).cuda()
        opt = FusedAdam(m.parameters(), lr=1e-3)
        g = torch.Generator(device="cuda").manual_seed(1)
        grads = []
        for _ in range(3):
            x = torch.rand(16, 3, 64, 64, device="cuda", generator=g)
            y = torch.randint(0, 10, (16,), device="cuda", generator=g)
            loss = cross_entropy(m(x), y)
            opt.zero_grad()
            loss.backward()
            grads.append(m._pvr_store.grad_flat.clone())  # read right after backward: must be complete
            opt.step(clip_norm=1.0)
        torch.cuda.synchronize()
        return grads, [p.detach().clone() for p in m.parameters()]

    ga, pa = run(True)
    gb, pb = run(False)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-6), (a - b).abs().max().item()
    for a, b in zip(pa, pb):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-5)


def _gloo_gpu_worker(rank, world, port, out_dir):
    """One rank of a 2-process DDP run whose ranks SHARE cuda:0 (gloo carries the gradients: RCCL
    needs one GPU per rank). Exercises the fused path's cross-rank bucket protocol exactly as a
    multi-GPU run does: weight gradients on the side stream, gradient-ready notifications, buckets
    launched in index order on every rank, end-of-backward join, all on a high-priority main stream."""
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    torch.manual_seed(100 + rank)  # different init per rank: the rank-0 broadcast must fix it
    m = ViT(**dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)).to(dev)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.1)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(4 * world, 3, 64, 64, generator=g)
    y = torch.randint(0, 10, (4 * world,), generator=g)
    xs, ys = x[4 * rank:4 * rank + 4].to(dev), y[4 * rank:4 * rank + 4].to(dev)
    main = torch.cuda.Stream(device=dev, priority=-1)
    main.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(main):
        for _ in range(2):  # the second step re-arms the buckets
            for p in m.parameters():
                if p.grad is not None:
                    p.grad.zero_()
            cross_entropy(ddp(xs), ys).backward()
    torch.cuda.synchronize()
    torch.save({"state": {k: v.detach().cpu().clone() for k, v in m.state_dict().items()},
                "grads": {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()},
                "nbuckets": len(ddp._buckets), "x": x, "y": y}, os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_two_ranks_fused_path_matches_single_process(tmp_path):
    import torch.multiprocessing as mp

    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy

    world = 2
    mp.spawn(_gloo_gpu_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"g{i}.pt", weights_only=True) for i in range(world)]
    assert r[0]["nbuckets"] > 2
    for k in r[0]["state"]:
        assert torch.equal(r[0]["state"][k], r[1]["state"][k]), f"params differ after broadcast: {k}"
    for n in r[0]["grads"]:
        assert torch.equal(r[0]["grads"][n], r[1]["grads"][n]), f"averaged gradient differs across ranks: {n}"
    dev = torch.device("cuda:0")
    ref = ViT(**dict(CFG, mlp_dropout=0.0, embedding_dropout=0.0)).to(dev)
    ref.load_state_dict(r[0]["state"])
    cross_entropy(ref(r[0]["x"].to(dev)), r[0]["y"].to(dev)).backward()
    torch.cuda.synchronize()
    for n, p in ref.named_parameters():
        a, b = r[0]["grads"][n].float(), p.grad.detach().cpu().float()
        err = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        assert err < 2e-2, f"{n}: DDP(2 ranks) vs single-process gradient rel err {err:.3e}"


def _gloo_gpu_recipe_worker(rank, world, port, out_dir, cfg, fp8, steps, poison_step, batch):
    """One rank of a 2-process DDP run sharing cuda:0 (gloo transport) with the full recipe: FusedAdam,
    clip 1.0, optionally fp8 GEMMs (per-rank delayed scaling) and a non-finite step on rank 1 only
    (its loss times Inf): the all-reduced gradients are then non-finite on BOTH ranks, so both skip."""
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    torch.manual_seed(100 + rank)  # different init per rank: the rank-0 broadcast must fix it
    m = ViT(**cfg).to(dev)
    if fp8:
        m.enable_fp8(wgrad=True)  # every fp8 GEMM kind, the opt-in weight gradients included
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.25)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(11 + rank)  # each rank its own data
    snaps, skipped, losses = [], [], []
    main = torch.cuda.Stream(device=dev, priority=-1)
    main.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(main):
        for step in range(steps):
            x = torch.rand(batch, 3, cfg["image_size"], cfg["image_size"], generator=g).to(dev)
            y = torch.randint(0, 10, (batch,), generator=g).to(dev)
            before = m._pvr_store.flat.clone() if step else None
            loss = cross_entropy(ddp(x), y)
            if step == poison_step and rank == 1:
                loss = loss * float("inf")
            opt.zero_grad()
            loss.backward()
            opt.step(clip_norm=1.0)
            torch.cuda.synchronize()
            losses.append(float(loss.item()))
            skipped.append(bool(before is not None and torch.equal(before, m._pvr_store.flat)))
            snaps.append(m._pvr_store.flat.detach().cpu().clone())
    torch.save({"snaps": snaps, "skipped": skipped, "losses": losses, "fp8_on": m._fp8 is not None,
                "grad_finite": bool(torch.isfinite(m._pvr_store.grad_flat).all().item())},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["fp8_nonfinite", "fp8_generic_attention"])
def test_ddp_two_ranks_recipe(case, tmp_path):
    """BASELINE configs 4-5 under data parallelism on the fused path: fp8 GEMMs (ViT-H/14's dtype) and
    a long sequence on the generic attention path (257 tokens: the in_proj bias gradient from column
    sums on the weight-gradient stream). Parameters stay bitwise identical across ranks after every
    step (each rank's fp8 scales are its own; the averaged gradients, hence the global-norm skip
    decision and the Adam update, are the same everywhere), and a step that overflows on one rank
    is skipped on both."""
    import torch.multiprocessing as mp

    if case == "fp8_nonfinite":
        cfg = dict(image_size=64, patch_size=16, num_transformer_layer=2, num_heads=2, embedding_dim=256, mlp_size=512,
                   num_classes=10, mlp_dropout=0.1, embedding_dropout=0.1)
        steps, poison, batch = 5, 2, 16  # 16 x 17 = 272 tokens: the fp8 path needs >= 256
    else:
        cfg = dict(image_size=64, patch_size=4, num_transformer_layer=2, num_heads=4, embedding_dim=256, mlp_size=512,
                   num_classes=10, mlp_dropout=0.1, embedding_dropout=0.1)
        steps, poison, batch = 3, -1, 4
    world = 2
    mp.spawn(_gloo_gpu_recipe_worker, args=(world, _free_port(), str(tmp_path), cfg, True, steps, poison, batch),
             nprocs=world, join=True)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert r[0]["fp8_on"] and r[1]["fp8_on"], "fp8 path did not engage"
    for s in range(steps):
        assert torch.equal(r[0]["snaps"][s], r[1]["snaps"][s]), f"parameters differ across ranks after step {s}"
    for i in range(world):
        for s in range(1, steps):
            assert r[i]["skipped"][s] == (s == poison), (case, i, r[i]["skipped"])
        assert r[i]["grad_finite"], "the step after the overflow must be finite again"
        assert all(v == v and abs(v) != float("inf") for s, v in enumerate(r[i]["losses"]) if s != poison)


def test_summary_on_gpu_model_matches_notebook():
    # torchinfo-style summary of a cuda model: the per-module path runs inside the summary (the fused
    # encoder would bypass the hooks), the fused path is back afterwards
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.utils.summary import summary

    m = ViT(num_classes=3).cuda()
    s = summary(m, input_size=(32, 3, 224, 224), print_out=False)
    assert s.total_params == 85_800_963 and f"{s.total_mult_adds / 1e9:.2f}" == "5.52"
    assert (s.input_mb, s.fwd_bwd_mb, s.params_mb, s.total_mb) == (19.27, 3330.74, 229.20, 3579.21)
    x = torch.randn(2, 3, 224, 224, device="cuda")
    assert _ext.use_fused(x)
    assert m(x).shape == (2, 3)


def test_device_prefetcher_copies_on_side_stream():
    """K17: the prefetcher's batches equal a blocking .to(device), land on the current device, and
    the engine consumes them (next batch's copy in flight on the copy stream)."""
    from torch.utils.data import DataLoader, TensorDataset

    from pytorch_vit_paper_replication_amd.data import DevicePrefetcher

    xs, ys = torch.randn(37, 3, 8, 8), torch.randint(0, 5, (37,))
    dl = DataLoader(TensorDataset(xs, ys), batch_size=8, pin_memory=True)
    pf = DevicePrefetcher(dl, "cuda")
    outs = [(x.clone(), y.clone()) for x, y in pf]
    torch.cuda.synchronize()
    assert len(outs) == 5 and all(x.is_cuda and y.is_cuda for x, y in outs)
    assert torch.equal(torch.cat([x for x, _ in outs]).cpu(), xs)
    assert torch.equal(torch.cat([y for _, y in outs]).cpu(), ys)
    # unpinned host tensors are pinned on the way (copy stays asynchronous)
    dl2 = DataLoader(TensorDataset(xs, ys), batch_size=16, pin_memory=False)
    assert torch.equal(torch.cat([x.cpu() for x, _ in DevicePrefetcher(dl2, "cuda")]), xs)


@pytest.mark.parametrize("fp8", [False, True])
def test_resume_is_bit_exact(fp8, tmp_path):
    """Checkpoint / resume on the fused path: 2 steps, save_checkpoint, a FRESH model + optimizer +
    scheduler, load_checkpoint, 2 more steps equals 4 uninterrupted steps bit for bit, with dropout
    on (the device dropout counter is saved) and in fp8 (the delayed-scaling histories are saved).
    Runs in deterministic mode (ordered reductions instead of float atomics), so that two runs of the
    same step are themselves bit-identical."""
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay
    from pytorch_vit_paper_replication_amd.utils.checkpoint import load_checkpoint, save_checkpoint

    cfg = dict(CFG, mlp_dropout=0.1, embedding_dropout=0.1)
    xs = [torch.rand(16, 3, 64, 64, device="cuda") for _ in range(4)]
    ys = [torch.randint(0, 10, (16,), device="cuda") for _ in range(4)]

    def make(seed):
        torch.manual_seed(seed)
        m = ViT(**cfg).cuda()
        if fp8:
            m.enable_fp8(wgrad=True)
        o = FusedAdam(param_groups_weight_decay(m, 0.03), lr=1e-3)
        return m, o, warmup_linear_decay(o, 10, 0.2)

    def run(m, o, s, steps):
        losses = []
        for i in steps:
            m.train()
            loss = cross_entropy(m(xs[i]), ys[i])
            o.zero_grad()
            loss.backward()
            o.step(clip_norm=1.0)
            s.step()
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
        return losses

    with _ext.deterministic_mode():
        _resume_check(make, run, fp8, tmp_path, save_checkpoint, load_checkpoint)


def _resume_check(make, run, fp8, tmp_path, save_checkpoint, load_checkpoint):
    ma, oa, sa = make(0)
    torch.manual_seed(123)
    la = run(ma, oa, sa, range(4))

    mb, ob, sb = make(0)
    torch.manual_seed(123)
    lb = run(mb, ob, sb, range(2))
    path = save_checkpoint(str(tmp_path), mb, ob, sb, epoch=1)
    del mb, ob, sb
    mc, oc, sc = make(1)  # different init: everything must come from the checkpoint
    load_checkpoint(str(path), mc, oc, sc)
    lb += run(mc, oc, sc, range(2, 4))
    if fp8:
        assert mc._fp8 is not None and all(mc._fp8.act.calibrated)
    for i, (a, b) in enumerate(zip(la, lb)):
        assert torch.equal(a, b), f"step {i}: loss {a.item()} vs {b.item()}"
    for (n, p1), p2 in zip(ma.named_parameters(), mc.parameters()):
        assert torch.equal(p1, p2), n
    assert torch.equal(oa._fused[1], oc._fused[1]) and torch.equal(oa._fused[2], oc._fused[2])


def test_odd_patch_size_fused_matches_reference():
    """Odd patch size (image 63, P 9: kc = 243 columns, not a multiple of 4): the fused patch
    embedding pads its weight with a plain zero pad and reduces the weight gradient through a
    temporary; forward and every gradient match the module-by-module PyTorch path."""
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy

    torch.manual_seed(0)
    cfg = dict(CFG, image_size=63, patch_size=9, embedding_dim=256, num_heads=4, mlp_size=512,
               mlp_dropout=0.0, embedding_dropout=0.0)
    mf, mr = ViT(**cfg).cuda(), ViT(**cfg).cuda()
    mr.load_state_dict(mf.state_dict())
    # 96 x 49 = 4704 patch rows, D = 256, K padded 243 -> 256: the patch weight gradient takes the
    # split-K ping-pong path, whose 16-B reduction cannot write 243 columns directly
    x = torch.rand(96, 3, 63, 63, device="cuda")
    y = torch.randint(0, 10, (96,), device="cuda")
    assert _ext.use_fused(x) and mf._fused_supported(x)
    lf = cross_entropy(mf(x), y)
    lf.backward()
    os.environ["PVR_DISABLE_FUSED"] = "1"
    try:
        lr_ = F.cross_entropy(mr(x).float(), y)
        lr_.backward()
    finally:
        os.environ["PVR_DISABLE_FUSED"] = "0"
    assert abs(lf.item() - lr_.item()) < 2e-2 * max(1.0, abs(lr_.item()))
    for (n, pf), pr in zip(mf.named_parameters(), mr.parameters()):
        g, gr = pf.grad.float(), pr.grad.float()
        rel = ((g - gr).norm() / gr.norm().clamp_min(1e-12)).item()
        assert rel < 5e-2, f"{n}: rel-L2 {rel:.3e}"


def test_deterministic_mode_gradients_bitwise_repeatable():
    """Deterministic mode at a size where the default reductions have many partial sums per element
    (4160 token rows: hundreds of LayerNorm-backward workgroups, 17 GEMM row tiles, 65 patch tokens):
    two backward passes of the same step give bit-identical gradients for every parameter."""
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy

    torch.manual_seed(0)
    m = ViT(**dict(CFG, image_size=128, embedding_dim=256, num_heads=4, mlp_size=1024, mlp_dropout=0.0,
                   embedding_dropout=0.0)).cuda()
    x = torch.rand(64, 3, 128, 128, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")

    def grads():
        m.zero_grad(set_to_none=False)
        cross_entropy(m(x), y).backward()
        torch.cuda.synchronize()
        return [p.grad.detach().clone() for p in m.parameters()]

    with _ext.deterministic_mode():
        assert _ext.ext().deterministic()
        g1, g2 = grads(), grads()
    assert not _ext.ext().deterministic()
    for (n, _), a, b in zip(m.named_parameters(), g1, g2):
        assert torch.equal(a, b), n


def test_deterministic_mode_long_sequence_attention_slabs():
    """Deterministic mode through the model at N = 401 (320 px / 16 + CLS = 256 + 145: two key blocks,
    neither the last-key nor the tail-split path), where the attention backward's dQ goes through
    per-key-block slabs summed in order: two backward passes give bit-identical gradients."""
    from pytorch_vit_paper_replication_amd import _ext
    from pytorch_vit_paper_replication_amd.models import ViT

    torch.manual_seed(0)
    m = ViT(**dict(CFG, image_size=320, embedding_dim=128, num_heads=2, mlp_size=256, mlp_dropout=0.0,
                   embedding_dropout=0.0)).cuda()
    x = torch.rand(4, 3, 320, 320, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")
    with _ext.deterministic_mode():
        g1, g2 = _grads(m, x, y), _grads(m, x, y)
    for (n, _), a, b in zip(m.named_parameters(), g1, g2):
        assert torch.equal(a, b), n
        assert torch.isfinite(a).all(), n


def _det_model_and_batch():
    from pytorch_vit_paper_replication_amd.models import ViT

    torch.manual_seed(0)
    m = ViT(**dict(CFG, image_size=128, embedding_dim=256, num_heads=4, mlp_size=1024, mlp_dropout=0.0,
                   embedding_dropout=0.0)).cuda()
    x = torch.rand(64, 3, 128, 128, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")
    return m, x, y


def _grads(m, x, y):
    from pytorch_vit_paper_replication_amd.ops.fused_vit import cross_entropy

    m.zero_grad(set_to_none=False)
    cross_entropy(m(x), y).backward()
    torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in m.parameters()]


def test_torch_deterministic_algorithms_covers_the_first_step():
    """torch.use_deterministic_algorithms(True) switched on before any fused backward (no
    deterministic_mode(), no env var): the native flag is synced at the first backward kernel
    (HeadFn.backward), so already the first step's gradients are bitwise repeatable."""
    from pytorch_vit_paper_replication_amd import _ext

    _ext.ext().set_deterministic(False)
    m, x, y = _det_model_and_batch()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        g1 = _grads(m, x, y)
        assert _ext.ext().deterministic()
        g2 = _grads(m, x, y)
    finally:
        torch.use_deterministic_algorithms(False)
    _grads(m, x, y)  # the next backward syncs the flag back off
    assert not _ext.ext().deterministic()
    for (n, _), a, b in zip(m.named_parameters(), g1, g2):
        assert torch.equal(a, b), n


def test_free_scratch_releases_and_recreates():
    """_ext.free_scratch() drops every per-stream scratch buffer (split-K workspaces, tail slabs,
    deterministic partial rows, attention scratch); the next step re-creates them and, in
    deterministic mode, reproduces the gradients bit for bit."""
    from pytorch_vit_paper_replication_amd import _ext

    m, x, y = _det_model_and_batch()
    with _ext.deterministic_mode():
        g1 = _grads(m, x, y)
        _ext.free_scratch()
        g2 = _grads(m, x, y)
    for (n, _), a, b in zip(m.named_parameters(), g1, g2):
        assert torch.equal(a, b), n
