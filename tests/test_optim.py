"""Optimizer recipe parity: FusedAdam (reference-math fallback) vs torch.optim.Adam, param groups,
warmup/decay schedule (MAIN.ipynb:2792-2960)."""
import torch

from pytorch_vit_paper_replication_amd.models import ViT
from pytorch_vit_paper_replication_amd.optim import FusedAdam, param_groups_weight_decay, warmup_linear_decay

SMALL = dict(image_size=32, patch_size=8, num_transformer_layer=2, num_heads=2, embedding_dim=32, mlp_size=64,
             num_classes=4)


def test_param_groups_counts_vit_b16():
    g = param_groups_weight_decay(ViT(num_classes=3), 0.03)
    assert len(g[0]["params"]) == 52 and sum(p.numel() for p in g[0]["params"]) == 85_678_848
    assert len(g[1]["params"]) == 100 and sum(p.numel() for p in g[1]["params"]) == 122_115
    assert g[0]["weight_decay"] == 0.03 and g[1]["weight_decay"] == 0.0


def test_fused_adam_matches_torch_adam_cpu():
    torch.manual_seed(0)
    a, b = ViT(**SMALL), ViT(**SMALL)
    b.load_state_dict(a.state_dict())
    oa = FusedAdam(param_groups_weight_decay(a, 0.03), lr=1e-2)
    ob = torch.optim.Adam(param_groups_weight_decay(b, 0.03), lr=1e-2, betas=(0.9, 0.999))
    for it in range(4):
        for pa, pb in zip(a.parameters(), b.parameters()):
            gr = torch.randn_like(pa) * (it + 1)
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        oa.step(clip_norm=1.0)
        torch.nn.utils.clip_grad_norm_(b.parameters(), 1.0)
        ob.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-6, rtol=1e-5)


def test_adamw_decoupled():
    torch.manual_seed(0)
    a, b = ViT(**SMALL), ViT(**SMALL)
    b.load_state_dict(a.state_dict())
    oa = FusedAdam(a.parameters(), lr=1e-2, weight_decay=0.1, decoupled_weight_decay=True)
    ob = torch.optim.AdamW(b.parameters(), lr=1e-2, weight_decay=0.1)
    for _ in range(3):
        for pa, pb in zip(a.parameters(), b.parameters()):
            gr = torch.randn_like(pa)
            pa.grad, pb.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-6, rtol=1e-5)


def test_warmup_linear_decay_matches_reference_schedule():
    """EPOCHS=10, 8 batches/epoch -> 80 steps, warmup 4, decay 76 (MAIN.ipynb cell 87 output)."""
    m = torch.nn.Linear(2, 2)
    o1 = torch.optim.Adam(m.parameters(), lr=1e-3)
    s1 = warmup_linear_decay(o1, 80, 0.05)
    o2 = torch.optim.Adam(m.parameters(), lr=1e-3)
    w = torch.optim.lr_scheduler.LinearLR(o2, start_factor=1e-6, end_factor=1, total_iters=4)
    d = torch.optim.lr_scheduler.LinearLR(o2, start_factor=1, end_factor=0, total_iters=76)
    s2 = torch.optim.lr_scheduler.SequentialLR(o2, schedulers=[w, d], milestones=[4])
    for _ in range(80):
        assert abs(o1.param_groups[0]["lr"] - o2.param_groups[0]["lr"]) < 1e-12
        o1.step(), o2.step()
        s1.step(), s2.step()
