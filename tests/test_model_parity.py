"""API / state_dict / numerics parity of models.vit with the reference."""
import inspect

import pytest
import torch

from models.vit import MLPBlock, MultiHeadSelfAttentionBlock, PatchEmbedding, TransformerEncoderBlock, ViT
from models import vit_no_classifier
from tests.refload import ref_module

SMALL = dict(image_size=32, patch_size=8, num_transformer_layer=2, num_heads=2, embedding_dim=64, mlp_size=128,
             num_classes=5)


def test_ctor_signature_and_defaults():
    sig = inspect.signature(ViT.__init__)
    defaults = {k: v.default for k, v in sig.parameters.items() if k != "self"}
    assert defaults == dict(image_size=224, patch_size=16, num_transformer_layer=12, num_heads=12, embedding_dim=768,
                            mlp_size=3072, attn_dropout=0, mlp_dropout=0.1, embedding_dropout=0.1, num_classes=1000)
    assert list(inspect.signature(PatchEmbedding.__init__).parameters)[1:] == [
        "image_size", "color_channels", "patch_size", "embedding_dropout", "embedding_dim"]
    assert list(inspect.signature(MultiHeadSelfAttentionBlock.__init__).parameters)[1:] == [
        "embedding_dim", "num_heads", "attn_dropout"]
    assert list(inspect.signature(MLPBlock.__init__).parameters)[1:] == ["embedding_dim", "mlp_size", "dropout"]
    assert list(inspect.signature(TransformerEncoderBlock.__init__).parameters)[1:] == [
        "embedding_dim", "num_heads", "attn_dropout", "mlp_size", "mlp_dropout"]


def test_param_counts_and_keys():
    m = ViT(num_classes=3)
    assert sum(p.numel() for p in m.parameters()) == 85_800_963  # MAIN.ipynb:2727
    assert sum(p.numel() for p in ViT().parameters()) == 86_567_656
    sd = m.state_dict()
    assert len(sd) == 152
    assert sd["transformer_encoder.0.msa_block.multi_head_attention.in_proj_weight"].shape == (2304, 768)
    assert sd["patch_embedding_block.position_embedding"].shape == (1, 197, 768)
    assert sd["classifier.0.weight"].shape == (3, 768)
    blk = TransformerEncoderBlock()
    assert sum(p.numel() for p in blk.parameters()) == 7_087_872  # MAIN.ipynb:2355


def test_state_dict_matches_reference_exactly_under_seed():
    ref = ref_module("models/vit.py", "ref_vit")
    torch.manual_seed(7)
    a = ViT(**SMALL)
    torch.manual_seed(7)
    b = ref.ViT(**SMALL)
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa) == list(sb)
    for k in sa:
        assert sa[k].shape == sb[k].shape, k
        assert torch.equal(sa[k], sb[k]), f"init differs for {k}"


def test_notebook_output_reproduced():
    """MAIN.ipynb cell 78 output: tensor([[ 0.6136, -0.9092,  0.5918]]) (set_seeds(); randn; ViT(3))."""
    from helper_functions import set_seeds

    set_seeds()
    x = torch.randn(1, 3, 224, 224)
    vit = ViT(num_classes=3)
    out = vit(x)
    assert torch.allclose(out, torch.tensor([[0.6136, -0.9092, 0.5918]]), atol=1e-4)


def test_forward_and_grad_parity_with_reference():
    ref = ref_module("models/vit.py", "ref_vit")
    torch.manual_seed(0)
    cfg = dict(SMALL, mlp_dropout=0.0, embedding_dropout=0.0)
    a = ViT(**cfg)
    b = ref.ViT(**cfg)
    b.load_state_dict(a.state_dict())
    x = torch.randn(3, 3, 32, 32)
    for m in (a, b):
        m.eval()
    assert torch.allclose(a(x), b(x), atol=1e-5)
    a.train()
    b.train()
    la, lb = a(x).logsumexp(1).sum(), b(x).logsumexp(1).sum()
    la.backward()
    lb.backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa.grad, pb.grad, atol=1e-5, rtol=1e-4), n


def test_reference_checkpoint_roundtrip(tmp_path):
    ref = ref_module("models/vit.py", "ref_vit")
    r = ref.ViT(**SMALL)
    p = tmp_path / "ref.pth"
    torch.save(r.state_dict(), p)
    a = ViT(**SMALL)
    a.load_state_dict(torch.load(p, weights_only=True), strict=True)
    r2 = ref.ViT(**SMALL)
    r2.load_state_dict(a.state_dict(), strict=True)
    x = torch.randn(2, 3, 32, 32)
    r.eval(), r2.eval()
    assert torch.allclose(r(x), r2(x))


@pytest.mark.parametrize("image_size,patch", [(224, 16), (384, 16), (64, 16)])
def test_output_shapes(image_size, patch):
    cfg = dict(image_size=image_size, patch_size=patch, num_transformer_layer=1, num_heads=2, embedding_dim=32,
               mlp_size=64)
    m = ViT(num_classes=7, **cfg).eval()
    x = torch.randn(2, 3, image_size, image_size)
    assert m(x).shape == (2, 7)
    b = vit_no_classifier.ViT(**cfg).eval()
    n = (image_size // patch) ** 2 + 1
    assert b(x).shape == (2, n, 32)


def test_no_classifier_state_dict_is_full_minus_head():
    full = set(ViT(**SMALL).state_dict())
    cfg = {k: v for k, v in SMALL.items() if k != "num_classes"}
    nc = set(vit_no_classifier.ViT(**cfg).state_dict())
    assert nc == {k for k in full if not k.startswith("classifier.")}
    ref = ref_module("models/vit_no_classifier.py", "ref_vit_nc")
    assert nc == set(ref.ViT(**cfg).state_dict())


def test_patch_size_assertion_message():
    with pytest.raises(AssertionError, match="Input image size must be divisible by patch size, image size: 250, patch_size: 16"):
        PatchEmbedding(image_size=250, patch_size=16)


def test_blocks_match_reference_blocks():
    ref = ref_module("models/vit.py", "ref_vit")
    torch.manual_seed(3)
    a = TransformerEncoderBlock(embedding_dim=64, num_heads=4, mlp_size=128, mlp_dropout=0.0)
    b = ref.TransformerEncoderBlock(embedding_dim=64, num_heads=4, mlp_size=128, mlp_dropout=0.0)
    b.load_state_dict(a.state_dict())
    x = torch.randn(2, 10, 64)
    assert torch.allclose(a(x), b(x), atol=1e-5)
    pe_a = PatchEmbedding(image_size=32, patch_size=8, embedding_dim=64, embedding_dropout=0.0)
    pe_b = ref.PatchEmbedding(image_size=32, patch_size=8, embedding_dim=64, embedding_dropout=0.0)
    pe_b.load_state_dict(pe_a.state_dict())
    img = torch.randn(2, 3, 32, 32)
    assert torch.allclose(pe_a(img), pe_b(img), atol=1e-6)
