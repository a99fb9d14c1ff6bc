"""CPU tests of the GEMM dispatch rules in ops/gemm.py (tile choice, weight-gradient split widths),
measured on MI355X in profiles/r5/tiles_12_13/ and profiles/r5/wgrad_width/."""
import pytest

from pytorch_vit_paper_replication_amd.ops import gemm as G


@pytest.fixture(autouse=True)
def _cus(monkeypatch):
    monkeypatch.setattr(G, "_n_cus", lambda: 256)  # an MI355X, whatever this host has
    monkeypatch.setattr(G, "FORCE_TILE", None)
    monkeypatch.setattr(G, "OVERLAPPED", False)


T_B16, T_L16 = 50432, 128 * 577


def test_persistent_kernel_for_short_k_with_four_tiles_per_cu():
    assert G._tile(T_B16, 2304, 768, "fwd") == 13          # qkv forward
    assert G._tile(T_B16, 3072, 768, "fwd") == 13          # fc1 forward (GELU epilogue)
    assert G._tile(T_B16, 3072, 768, "dgrad_t") == 13      # fc2 dgrad (dGELU epilogue; since round 5)
    assert G._tile(T_B16, 768, 3072, "fwd") == 12          # fc2 forward: 2.3 tiles per CU
    assert G._tile(T_L16, 1024, 1024, "fwd") == 13          # ViT-L/16-384 out-projection


def test_long_k_stays_on_one_tile_per_workgroup():
    assert G._tile(T_L16, 1024, 4096, "fwd") == 12          # ViT-L/16-384 fc2 forward (K 4096)
    assert G._tile(T_L16, 1024, 3072, "dgrad_t") == 12      # qkv dgrad (K 3072)


def test_wgrad_split_width_narrow_only_beside_the_main_stream():
    # ViT-B/16 qkv weight (2304 x 768, 27 tiles): a full wave (9 splits) on a serial schedule,
    # ~144 workgroups (5 splits) on the side stream
    assert G.wgrad_splits(T_B16, 2304, 768, 12) == 9
    G.OVERLAPPED = True
    assert G.wgrad_splits(T_B16, 2304, 768, 12) == 5
    assert G.wgrad_splits(T_B16, 3072, 768, 12) == 4
    # wide weights (ViT-H/14 qkv 3840 x 1280, 75 tiles) keep the full wave either way
    assert G.wgrad_splits(256 * 257, 3840, 1280, 12) == 3
