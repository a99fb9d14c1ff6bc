"""Data-parallel logic on CPU: 2-8 gloo ranks (torch.multiprocessing), SURVEY.md §4.3 item 3.

* rank-dependent init is overwritten by the rank-0 broadcast (C1),
* bucketed, backward-overlapped gradient averaging equals single-process gradients on the
  concatenated batch (C2), including with several small buckets,
* engine.train under DDP reduces metrics across ranks (C4) so every rank returns the same results.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CFG = dict(image_size=32, patch_size=8, num_transformer_layer=2, num_heads=2, embedding_dim=32, mlp_size=64,
           num_classes=5, mlp_dropout=0.0, embedding_dropout=0.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, bucket_mb, wire=None):
    os.environ["PVR_DISABLE_FUSED"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = ViT(**CFG)
    ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_mb,
                                  comm_dtype=getattr(torch, wire) if wire else None)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2 * world, 3, 32, 32, generator=g)
    y = torch.randint(0, 5, (2 * world,), generator=g)
    xs, ys = x[2 * rank:2 * rank + 2], y[2 * rank:2 * rank + 2]
    for _ in range(2):  # two iterations: buckets must re-arm
        for p in model.parameters():
            p.grad = None
        loss = torch.nn.functional.cross_entropy(ddp(xs), ys)
        loss.backward()
    torch.save({"state": {k: v.clone() for k, v in model.state_dict().items()},
                "grads": {n: p.grad.clone() for n, p in model.named_parameters()},
                "nbuckets": len(ddp._buckets), "x": x, "y": y}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def _rel_l2(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ddp_bf16_wire_grads_track_fp32(tmp_path, world):
    """bf16 wire format (persistent bf16 mirror of the fp32 gradient buckets): the averaged gradients
    stay within bf16 rounding of the single-process fp32 gradients and agree bit-for-bit across ranks."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), 0.01, "bfloat16"), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    from pytorch_vit_paper_replication_amd.models import ViT

    ref = ViT(**CFG)
    ref.load_state_dict(r[0]["state"])
    torch.nn.functional.cross_entropy(ref(r[0]["x"]), r[0]["y"]).backward()
    worst = 0.0
    for n, p in ref.named_parameters():
        e = _rel_l2(r[0]["grads"][n], p.grad)
        worst = max(worst, e)
        # bf16 keeps 8 mantissa bits: one rounding of every rank's gradient plus the (world - 1)
        # bf16 partial sums of the reduction -> rel-L2 well under 1e-2
        assert e < 1e-2, (n, e)
        for i in range(1, world):
            assert torch.equal(r[0]["grads"][n], r[i]["grads"][n]), f"{n} (rank {i})"
    print(f"bf16 wire, world {world}: worst per-tensor rel-L2 vs fp32 = {worst:.2e}")


@pytest.mark.parametrize("world,bucket_mb", [(2, 25.0), (2, 0.01), (4, 0.01), (8, 0.05)])
def test_ddp_grads_match_single_process(tmp_path, world, bucket_mb):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), bucket_mb), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    if bucket_mb < 1:
        assert r[0]["nbuckets"] > (5 if bucket_mb <= 0.01 else 1)
    for k in r[0]["state"]:
        for i in range(1, world):
            assert torch.equal(r[0]["state"][k], r[i]["state"][k]), f"params differ after broadcast: {k} (rank {i})"
    from pytorch_vit_paper_replication_amd.models import ViT

    ref = ViT(**CFG)
    ref.load_state_dict(r[0]["state"])
    loss = torch.nn.functional.cross_entropy(ref(r[0]["x"]), r[0]["y"])
    loss.backward()
    for n, p in ref.named_parameters():
        assert torch.allclose(r[0]["grads"][n], p.grad, atol=1e-6, rtol=1e-4), n
        for i in range(1, world):
            assert torch.equal(r[0]["grads"][n], r[i]["grads"][n]), f"{n} (rank {i})"


def _engine_worker(rank, world, port, out_dir):
    os.environ["PVR_DISABLE_FUSED"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from pytorch_vit_paper_replication_amd import engine
    from pytorch_vit_paper_replication_amd.data import create_synthetic_dataloaders
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    tr, te, _ = create_synthetic_dataloaders(batch_size=2, train_len=8, test_len=4, image_size=32, num_classes=5)
    model = ViT(**CFG)
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.05, timing=True)
    opt = FusedAdam(param_groups_weight_decay(model, 0.03), lr=1e-3)
    sched = warmup_linear_decay(opt, 2 * len(tr))
    res = engine.train(ddp, tr, te, opt, torch.nn.CrossEntropyLoss(), sched, epochs=2, device="cpu",
                       step_metrics_path=os.path.join(out_dir, "steps.jsonl"), log_every=3)
    torch.save({"res": res, "w": model.classifier[0].weight.detach().clone()}, os.path.join(out_dir, f"e{rank}.pt"))
    dist.destroy_process_group()


def test_engine_under_ddp_consistent_across_ranks(tmp_path):
    world = 2
    mp.spawn(_engine_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    a, b = (torch.load(tmp_path / f"e{i}.pt", weights_only=True) for i in range(world))
    assert a["res"] == b["res"]
    assert torch.equal(a["w"], b["w"]), "replicas diverged"
    # per-step JSONL from rank 0 only: 2 epochs x (8 images / 2 ranks / batch 2) = 4 steps
    import json

    from pytorch_vit_paper_replication_amd.utils.metrics import StepLogger

    recs = [json.loads(ln) for ln in open(tmp_path / "steps.jsonl")]
    assert [r["step"] for r in recs] == [0, 1, 2, 3] and [r["epoch"] for r in recs] == [0, 0, 1, 1]
    for r in recs:
        assert set(r) == set(StepLogger.SCHEMA) and r["kind"] == "step"
        assert r["world"] == 2 and r["rank"] == 0 and r["batch"] == 2
        assert r["ms"] > 0 and r["img_s"] > 0 and r["lr"] > 0
        assert r["grad_norm"] > 0 and r["loss"] > 0
        assert len(r["allreduce"]) > 1 and r["allreduce_ms"] >= 0
        # buckets padded to world x 7 x 4 KiB
        assert all(x["bytes"] % (2 * 7 * 4096) == 0 for x in r["allreduce"])


def test_embedding_gets_a_small_final_bucket():
    """The first-registered parameters (class token, position embedding, patch conv) receive their
    gradients last: they must sit in a small bucket of their own, so the first encoder block's bucket
    is all-reduced while the embedding backward runs and only a few MB remain after backward."""
    from pytorch_vit_paper_replication_amd.models import vit
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        m = vit("vit_b16")
        ddp = DistributedDataParallel(m, bucket_cap_mb=28.0)
        st = ddp._setup(torch.device("cpu"))
        names = {id(p): n for n, p in m.named_parameters()}
        last = {names[id(st.params[i])] for i in ddp._buckets[-1][2]}
        lo, hi, _ = ddp._buckets[-1]
        assert (hi - lo) * 4 <= 4 << 20
        assert {"patch_embedding_block.class_token", "patch_embedding_block.position_embedding",
                "patch_embedding_block.patch_and_flatten.0.weight"} <= last
        before = {names[id(st.params[i])] for i in ddp._buckets[-2][2]}
        assert not any(n.startswith("patch_embedding_block") for n in before)
        # buckets tile the flat gradient buffer exactly, in reverse registration order
        spans = sorted((lo, hi) for lo, hi, _ in ddp._buckets)
        assert spans[0][0] == 0 and spans[-1][1] == st.numel
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 8])
def test_bucket_layout_is_padded_to_world_x_7_x_4kib(world):
    """Every bucket is a contiguous flat range whose size is a multiple of world x 7 x 4 KiB; the
    buckets tile the gradient buffer; parameters keep their values across the re-layout."""
    from pytorch_vit_paper_replication_amd.models import vit
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel
    from pytorch_vit_paper_replication_amd.runtime.param_store import get_store

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        m = vit("vit_b16", num_classes=10)
        before = {n: p.detach().clone() for n, p in m.named_parameters()}
        get_store(m, torch.device("cpu"))  # an unpadded store exists first: DDP must re-lay it out
        ddp = DistributedDataParallel(m, bucket_cap_mb=28.0)
        ddp.world = world  # layout arithmetic only (the group has one rank)
        st = ddp._setup(torch.device("cpu"))
        quantum = world * 7 * 4096
        assert st.layout is not None and st.layout[1] * 4 == quantum
        for lo, hi, idxs in ddp._buckets:
            assert ((hi - lo) * 4) % quantum == 0 and (lo * 4) % quantum == 0
            for i in idxs:  # every member lies inside its bucket
                assert lo <= st.offsets[i] and st.offsets[i] + st.params[i].numel() <= hi
        spans = sorted((lo, hi) for lo, hi, _ in ddp._buckets)
        assert spans[0][0] == 0 and spans[-1][1] == st.numel
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        pad = st.numel - sum((p.numel() + 63) // 64 * 64 for p in st.params)
        assert 0 <= pad < len(ddp._buckets) * st.layout[1]
        for n, p in m.named_parameters():
            assert torch.equal(p.detach(), before[n]), n
            assert p.data.data_ptr() == st.flat[st.offset(p):].data_ptr()
    finally:
        dist.destroy_process_group()
