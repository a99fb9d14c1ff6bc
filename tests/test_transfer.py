"""Transfer-learning utilities, the nn.TransformerEncoder prototype and notebook scaffolding
(SURVEY.md §2.1 #20-#22). torchvision checkpoints are not available here: the key mapping is
pinned with synthetic state dicts in torchvision's naming (parity against real weights unpinned)."""
import pytest
import torch

from pytorch_vit_paper_replication_amd.models import (PatchEmbeddingV1, ViT, ViTTorchEncoder, feature_extractor,
                                                      from_torchvision_state_dict, to_torchvision_state_dict,
                                                      vit_from_torchvision_checkpoint)
from pytorch_vit_paper_replication_amd.models.transfer import set_layernorm_eps

TINY = dict(image_size=32, patch_size=8, num_transformer_layer=2, num_heads=2, embedding_dim=32, mlp_size=64,
            num_classes=5)


def test_torchvision_mapping_roundtrip_and_checkpoint(tmp_path):
    torch.manual_seed(0)
    m = set_layernorm_eps(ViT(**TINY), 1e-6).eval()
    tv = to_torchvision_state_dict(m.state_dict())
    assert "encoder.layers.encoder_layer_1.self_attention.in_proj_weight" in tv
    assert "conv_proj.weight" in tv and "encoder.pos_embedding" in tv and "heads.head.weight" in tv
    back = from_torchvision_state_dict(tv)
    assert set(back) == set(m.state_dict())
    p = tmp_path / "tv_vit.pth"
    torch.save(tv, p)
    m2 = vit_from_torchvision_checkpoint(str(p), num_heads=2).eval()
    assert m2.config["image_size"] == 32 and m2.config["num_transformer_layer"] == 2
    assert all(ln.eps == 1e-6 for ln in m2.modules() if isinstance(ln, torch.nn.LayerNorm))
    x = torch.rand(2, 3, 32, 32)
    with torch.no_grad():
        assert torch.allclose(m(x), m2(x), atol=1e-6)


def test_torchvision_legacy_mlp_names():
    m = ViT(**TINY)
    tv = {k.replace("mlp.0.", "mlp.linear_1.").replace("mlp.3.", "mlp.linear_2."): v
          for k, v in to_torchvision_state_dict(m.state_dict()).items()}
    assert set(from_torchvision_state_dict(tv)) == set(m.state_dict())
    with pytest.raises(KeyError):
        from_torchvision_state_dict({"encoder.bogus": torch.zeros(1)})


def test_feature_extractor_trains_head_only():
    from going_modular import engine
    from pytorch_vit_paper_replication_amd.optim import FusedAdam

    torch.manual_seed(0)
    m = feature_extractor(ViT(**TINY), num_classes=3, seed=0)
    trainable = [n for n, p in m.named_parameters() if p.requires_grad]
    assert trainable == ["classifier.0.weight", "classifier.0.bias"]
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == 32 * 3 + 3
    frozen = {n: p.detach().clone() for n, p in m.named_parameters() if not p.requires_grad}
    x, y = torch.rand(8, 3, 32, 32), torch.randint(0, 3, (8,))
    dl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=4)
    opt = FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0)
    res = engine.train(m, dl, dl, opt, torch.nn.CrossEntropyLoss(), sched, epochs=2, device="cpu")
    assert len(res["train_loss"]) == 2
    for n, p in m.named_parameters():
        if n in frozen:
            assert torch.equal(p, frozen[n]), n


def test_torch_encoder_prototype_matches_vit():
    torch.manual_seed(0)
    proto = ViTTorchEncoder(**TINY).eval()
    assert len(proto.transformer_encoder.layers) == 2
    assert len(ViTTorchEncoder(**dict(TINY, num_heads=4), replicate_num_layers_bug=True).transformer_encoder.layers) == 4
    vit = proto.to_vit().eval()
    assert sum(p.numel() for p in vit.parameters()) == sum(p.numel() for p in proto.parameters())
    x = torch.rand(3, 3, 32, 32)
    with torch.no_grad():
        assert torch.allclose(proto(x), vit(x), atol=1e-5)
    proto2 = ViTTorchEncoder(**TINY).from_vit(vit).eval()
    with torch.no_grad():
        assert torch.allclose(proto2(x), vit(x), atol=1e-5)


def test_torch_encoder_param_count_reference():
    # EX.ipynb:662: 85,800,963 parameters for ViT-B/16 with 3 classes, same as the custom ViT
    m = ViTTorchEncoder(num_classes=3)
    assert sum(p.numel() for p in m.parameters()) == 85_800_963


def test_patch_embedding_v1():
    pe = PatchEmbeddingV1(in_channels=3, patch_size=16, embedding_dim=768)
    assert pe(torch.rand(1, 3, 224, 224)).shape == (1, 196, 768)
    with pytest.raises(AssertionError, match="divisble by patch size"):
        pe(torch.rand(1, 3, 250, 250))
