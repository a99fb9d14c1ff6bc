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


def _worker(rank, world, port, out_dir, bucket_mb):
    os.environ["PVR_DISABLE_FUSED"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from pytorch_vit_paper_replication_amd.models import ViT
    from pytorch_vit_paper_replication_amd.parallel import DistributedDataParallel

    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = ViT(**CFG)
    ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_mb)
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
    ddp = DistributedDataParallel(model)
    opt = FusedAdam(param_groups_weight_decay(model, 0.03), lr=1e-3)
    sched = warmup_linear_decay(opt, 2 * len(tr))
    res = engine.train(ddp, tr, te, opt, torch.nn.CrossEntropyLoss(), sched, epochs=2, device="cpu")
    torch.save({"res": res, "w": model.classifier[0].weight.detach().clone()}, os.path.join(out_dir, f"e{rank}.pt"))
    dist.destroy_process_group()


def test_engine_under_ddp_consistent_across_ranks(tmp_path):
    world = 2
    mp.spawn(_engine_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    a, b = (torch.load(tmp_path / f"e{i}.pt", weights_only=True) for i in range(world))
    assert a["res"] == b["res"]
    assert torch.equal(a["w"], b["w"]), "replicas diverged"


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
