"""The CLI trainer (the reference's GM/train.py, which raised TypeError for lack of an LR scheduler,
SURVEY.md §2.1 #13): synthetic ViT and ImageFolder TinyVGG runs end to end on CPU, plus resume."""
import os

import numpy as np
import torch
from PIL import Image

from pytorch_vit_paper_replication_amd.cli.train import main


def test_cli_synthetic_vit(tmp_path, capsys):
    rc = main(["--model", "vit_tiny_test", "--synthetic", "--epochs", "1", "--batch-size", "4", "--image-size", "32",
               "--num-classes", "3", "--synthetic-train-len", "8", "--synthetic-test-len", "4",
               "--save-dir", str(tmp_path), "--save-name", "v.pth", "--checkpoint-dir", str(tmp_path / "ck"),
               "--metrics", str(tmp_path / "m.jsonl")])
    assert rc == 0
    sd = torch.load(tmp_path / "v.pth", weights_only=True)
    assert "classifier.0.weight" in sd and sd["classifier.0.weight"].shape[0] == 3
    assert (tmp_path / "m.jsonl").exists()
    ck = sorted(os.listdir(tmp_path / "ck"))
    assert ck, "no checkpoint written"
    capsys.readouterr()
    # --epochs is the total: the resumed run trains epoch 2 only, numbered 2
    rc = main(["--model", "vit_tiny_test", "--synthetic", "--epochs", "2", "--batch-size", "4", "--image-size", "32",
               "--num-classes", "3", "--synthetic-train-len", "8", "--synthetic-test-len", "4",
               "--save-dir", str(tmp_path), "--save-name", "v2.pth", "--resume", str(tmp_path / "ck" / ck[-1])])
    assert rc == 0
    out = capsys.readouterr().out
    assert "Epoch: 2 |" in out and "Epoch: 1 |" not in out, out


def test_cli_imagefolder_tinyvgg(tmp_path):
    rng = np.random.default_rng(0)
    for split in ("train", "test"):
        for cls in ("pizza", "steak", "sushi"):
            d = tmp_path / "data" / split / cls
            d.mkdir(parents=True)
            for i in range(2):
                Image.fromarray(rng.integers(0, 255, (80, 70, 3), dtype=np.uint8)).save(d / f"{i}.jpg")
    rc = main(["--model", "tinyvgg", "--train-dir", str(tmp_path / "data" / "train"), "--test-dir",
               str(tmp_path / "data" / "test"), "--image-size", "64", "--epochs", "1", "--batch-size", "3",
               "--num-workers", "0", "--save-dir", str(tmp_path), "--save-name", "t.pth"])
    assert rc == 0
    assert (tmp_path / "t.pth").exists()


def test_cli_fp8_and_options(tmp_path, monkeypatch):
    """--dtype fp8 / --fp8-grad / --dropout / --deterministic reach the model and the run (on the CPU the
    fused fp8 path does not engage: the reference math runs, the configuration is still recorded)."""
    from pytorch_vit_paper_replication_amd.cli import train as T
    from pytorch_vit_paper_replication_amd.models import presets

    made = []
    orig = presets.vit

    def spy(*a, **kw):
        m = orig(*a, **kw)
        made.append(m)
        return m

    monkeypatch.setattr("pytorch_vit_paper_replication_amd.models.vit", spy)
    rc = T.main(["--model", "vit_tiny_test", "--synthetic", "--epochs", "1", "--batch-size", "4", "--image-size", "32",
                 "--num-classes", "3", "--synthetic-train-len", "8", "--synthetic-test-len", "4", "--save-dir", str(tmp_path),
                 "--dtype", "fp8", "--fp8-grad", "e5m2", "--dropout", "0.0", "--deterministic"])
    assert rc == 0 and made
    m = made[0]
    assert m._fp8_cfg is not None and m._fp8_cfg[3] is True and m._fp8_cfg[4] == "e5m2"
    assert all(mod.p == 0.0 for mod in m.modules() if isinstance(mod, torch.nn.Dropout))
    a = T.build_parser().parse_args([])
    assert a.dtype == "bf16" and a.fp8_grad == "e4m3" and a.comm_dtype == "fp32" and not a.deterministic
