"""CPU tests of the auxiliary API surface: torchinfo-style summary (MAIN.ipynb:2317-2322), transforms
(MAIN.ipynb:254-265, EX.ipynb:225-232, GM/predictions.py:46-54), single-image prediction
(GM/predictions.py:20-83), plot_loss_curves / download_data / set_seeds (the course helper_functions,
MAIN.ipynb:81), JSONL metrics and ROCTX ranges."""
import json
import os
import re

import numpy as np
import pytest
import torch
from PIL import Image

from pytorch_vit_paper_replication_amd.data import transforms as T
from pytorch_vit_paper_replication_amd.models import ViT
from pytorch_vit_paper_replication_amd.utils.metrics import StepTimer, WallTimer, append_jsonl
from pytorch_vit_paper_replication_amd.utils.profiling import range_push
from pytorch_vit_paper_replication_amd.utils.summary import count_params, summary


def _img(w=40, h=30, seed=0):
    rng = np.random.default_rng(seed)
    return Image.fromarray(rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8), "RGB")


def test_vit_b16_param_count_matches_reference():
    # EX.ipynb:662 / MAIN.ipynb torchinfo output: ViT-B/16 with 3 classes has 85,800,963 params
    m = ViT(num_classes=3)
    assert count_params(m) == 85_800_963
    assert count_params(m, trainable_only=True) == 85_800_963


def test_summary_small_vit_reports_totals_and_shapes():
    m = ViT(image_size=32, patch_size=16, num_transformer_layer=2, num_heads=2, embedding_dim=32, mlp_size=64,
            num_classes=5)
    s = summary(m, input_size=(2, 3, 32, 32), depth=1, print_out=False)
    assert f"Total params: {count_params(m):,}" in s
    assert "Non-trainable params: 0" in s
    assert "[2, 5]" in s  # classifier output shape
    for p in m.patch_embedding_block.parameters():
        p.requires_grad_(False)
    s2 = summary(m, input_size=(2, 3, 32, 32), depth=1, print_out=False)
    frozen = sum(p.numel() for p in m.patch_embedding_block.parameters())
    assert f"Non-trainable params: {frozen:,}" in s2
    assert m.training  # summary restores the train flag


def test_resize_totensor_normalize():
    img = _img(40, 30)
    x = T.Compose([T.Resize((24, 20)), T.ToTensor()])(img)
    assert x.shape == (3, 24, 20) and x.dtype == torch.float32
    assert 0.0 <= x.min().item() and x.max().item() <= 1.0
    # int size resizes the short side, keeping the aspect ratio
    assert T.Resize(15)(img).size == (20, 15)
    # Normalize is (x - mean) / std per channel
    n = T.Normalize()(x)
    mean = torch.tensor(T.IMAGENET_MEAN).view(3, 1, 1)
    std = torch.tensor(T.IMAGENET_STD).view(3, 1, 1)
    torch.testing.assert_close(n, (x - mean) / std)


def test_v2_pipeline_matches_totensor():
    img = _img(16, 16, seed=1)
    a = T.default_vit_transform(16)(img)
    b = T.ToTensor()(img)
    torch.testing.assert_close(a, b)  # same-size resize is the identity; scale=True maps to [0,1]
    u8 = T.ToImage()(img)
    assert u8.dtype == torch.uint8 and u8.shape == (3, 16, 16)
    assert T.ToDtype(torch.float32, scale=False)(u8).max().item() > 1.0


def test_center_crop_pil_and_tensor_agree():
    img = _img(40, 30, seed=2)
    crop_pil = T.ToTensor()(T.CenterCrop(20)(img))
    crop_t = T.CenterCrop(20)(T.ToTensor()(img))
    assert crop_pil.shape == (3, 20, 20)
    torch.testing.assert_close(crop_pil, crop_t)
    y = T.imagenet_eval_transform(image_size=24, resize=32)(img)
    assert y.shape == (3, 24, 24)


def test_tensor_resize_keeps_uint8():
    t = torch.randint(0, 256, (3, 10, 12), dtype=torch.uint8)
    r = T.Resize((5, 6))(t)
    assert r.dtype == torch.uint8 and r.shape == (3, 5, 6)


def test_predict_and_plot(tmp_path):
    from pytorch_vit_paper_replication_amd.predictions import pred_and_plot_image, predict_image

    path = tmp_path / "img.jpg"
    _img(50, 40, seed=3).save(path)
    torch.manual_seed(0)
    m = ViT(image_size=32, patch_size=16, num_transformer_layer=1, num_heads=2, embedding_dim=32, mlp_size=64,
            num_classes=3)
    label, probs, _ = predict_image(m, str(path), image_size=(32, 32), device="cpu")
    assert probs.shape == (1, 3) and 0 <= label < 3
    torch.testing.assert_close(probs.sum(), torch.tensor(1.0))
    assert label == int(probs.argmax())
    out = tmp_path / "pred.png"
    assert pred_and_plot_image(m, ["a", "b", "c"], str(path), image_size=(32, 32), device="cpu",
                               save_path=str(out)) is None
    assert out.is_file() and out.stat().st_size > 0


def test_helper_functions(tmp_path, monkeypatch):
    import helper_functions as hf

    res = {"train_loss": [1.0, 0.5], "test_loss": [1.1, 0.7], "train_acc": [0.3, 0.6], "test_acc": [0.2, 0.5]}
    out = tmp_path / "curves.png"
    hf.plot_loss_curves(res, save_path=str(out))
    assert out.is_file() and out.stat().st_size > 0

    monkeypatch.chdir(tmp_path)
    (tmp_path / "data" / "pizza_steak_sushi").mkdir(parents=True)
    assert hf.download_data("http://unused", "pizza_steak_sushi").name == "pizza_steak_sushi"
    with pytest.raises(RuntimeError, match="No network"):
        hf.download_data("http://unused", "missing_dataset")

    hf.set_seeds(7)
    a = torch.rand(3)
    hf.set_seeds(7)
    torch.testing.assert_close(a, torch.rand(3))


def test_metrics_jsonl_and_timers(tmp_path):
    p = tmp_path / "m.jsonl"
    append_jsonl(str(p), {"step": 1, "loss": 2.5})
    append_jsonl(str(p), {"step": 2, "loss": 2.0})
    recs = [json.loads(line) for line in p.read_text().splitlines()]
    assert recs == [{"step": 1, "loss": 2.5}, {"step": 2, "loss": 2.0}]
    t = StepTimer()
    t.mark()
    t.mark()
    if not torch.cuda.is_available():
        assert t.intervals_ms() == []
    with WallTimer() as w:
        sum(range(1000))
    assert w.elapsed >= 0.0


def test_range_push_is_transparent(monkeypatch):
    for flag in ("0", "1"):  # with PVR_ROCTX=1 it pushes/pops a ROCTX range if libroctx64 loads
        monkeypatch.setenv("PVR_ROCTX", flag)
        with range_push("fwd"):
            x = 1 + 1
        assert x == 2


def test_summary_matches_notebook_torchinfo_figures():
    # MAIN.ipynb cell 80 / EX.ipynb cell 17: torchinfo.summary(ViT(num_classes=3), (32, 3, 224, 224))
    torch.manual_seed(0)
    s = summary(ViT(num_classes=3), input_size=(32, 3, 224, 224), print_out=False)
    assert s.total_params == 85_800_963 and s.trainable_params == 85_800_963
    assert f"{s.total_mult_adds / 1e9:.2f}" == "5.52"
    assert (s.input_mb, s.fwd_bwd_mb, s.params_mb, s.total_mb) == (19.27, 3330.74, 229.20, 3579.21)
    text = str(s)
    for row in ("PatchEmbedding (patch_embedding_block)", "MultiHeadSelfAttentionBlock (msa_block)",
                "Conv2d (0)", "Linear (0)"):
        assert row in text
    lines = {re.split(r"\s{2,}", ln.lstrip("│ └├─"))[0]: ln for ln in text.splitlines()}
    assert "152,064" in lines["PatchEmbedding (patch_embedding_block)"]
    assert "590,592" in lines["Conv2d (0)"]
    assert "2,363,904" in lines["MultiHeadSelfAttentionBlock (msa_block)"]
    assert "4,723,968" in lines["MLPBlock (mlp_block)"]
    assert "2,307" in lines["Linear (0)"] and "[32, 3]" in lines["Linear (0)"]


def test_summary_encoder_block_and_frozen_rows():
    # MAIN.ipynb cell 71: the encoder block alone, batch 1 -> 7,087,872 params, 4.73 M mult-adds,
    # 0.61 / 8.47 / 18.90 / 27.98 MB; the attention row carries nn.MultiheadAttention's 2,362,368
    from pytorch_vit_paper_replication_amd.models.vit import TransformerEncoderBlock
    blk = TransformerEncoderBlock()
    s = summary(blk, input_size=(1, 197, 768), print_out=False)
    assert s.total_params == 7_087_872
    assert f"{s.total_mult_adds / 1e6:.2f}" == "4.73"
    assert (s.input_mb, s.fwd_bwd_mb, s.params_mb, s.total_mb) == (0.61, 8.47, 18.90, 27.98)
    att = [ln for ln in str(s).splitlines() if "(multi_head_attention)" in ln][0]
    assert "2,362,368" in att and "--" in att  # keyword-called: no input shape, like torchinfo
    for p in blk.mlp_block.parameters():
        p.requires_grad_(False)
    s2 = str(summary(blk, input_size=(1, 197, 768), print_out=False))
    mlp = [ln for ln in s2.splitlines() if "Linear (0)" in ln][0]
    assert "(2,362,368)" in mlp and "False" in mlp
    top = s2.splitlines()[3]
    assert "Partial" in top


def test_device_prefetcher_cpu_passthrough():
    """K17 prefetcher: on a CPU device it yields the loader's batches unchanged, keeps len() and
    the sampler reachable (DistributedSampler.set_epoch), and is a no-op wrapper for prefetch()."""
    from torch.utils.data import DataLoader, TensorDataset

    from pytorch_vit_paper_replication_amd.data import DevicePrefetcher, prefetch

    xs, ys = torch.randn(10, 3, 4, 4), torch.arange(10)
    dl = DataLoader(TensorDataset(xs, ys), batch_size=4)
    assert prefetch(dl, "cpu") is dl
    pf = DevicePrefetcher(dl, "cpu")
    assert len(pf) == 3 and pf.sampler is dl.sampler and pf.dataset is dl.dataset
    got = list(pf)
    assert len(got) == 3
    assert torch.equal(torch.cat([b[0] for b in got]), xs) and torch.equal(torch.cat([b[1] for b in got]), ys)
    assert list(pf)[0][0].shape == (4, 3, 4, 4)  # re-iterable
