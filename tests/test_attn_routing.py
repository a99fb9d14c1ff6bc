"""Host-side routing of the attention backward for the BASELINE model shapes (CPU: the extension's
planning entry points run without a GPU).

* ViT-B/16 (N 197, dh 64): the pipelined whole-head kernel, in_proj bias partials per 32-query block.
* ViT-H/14 (N 257 = 256 + 1, dh 80) and ViT-L/16 at 384 px (N 577 = 2 x 256 + 65, dh 64): the
  generic kernels write every final dQ value (last-key pre-pass / f32 dQ slabs), so they emit one
  bias-partial row per (batch, head) and can write dQKV's e5m2 copy themselves.
* Attention dropout: no bias partials (rows of the dropped P do not sum to 1).
* N = 513 (three key blocks, 1-key tail): f32 atomics + conversion pass, so neither.
"""
import pytest

from pytorch_vit_paper_replication_amd import _ext

pytestmark = pytest.mark.skipif(not _ext.available(), reason="extension not built")


@pytest.mark.parametrize("B,N,H,D,drop,rows,q8", [
    (256, 197, 12, 768, False, 7, False),    # ViT-B/16: pipelined kernel
    (256, 257, 16, 1280, False, 1, True),    # ViT-H/14: lastkey path
    (256, 257, 16, 1280, True, 0, False),    # ... with attention dropout
    (128, 577, 16, 1024, False, 1, True),    # ViT-L/16 @ 384: slab path
    (128, 577, 16, 1024, True, 0, True),     # ... with dropout: slabs still write the final dQ
    (4, 513, 4, 256, False, 0, False),       # three key blocks + 1 key: atomics
])
def test_attn_bwd_routing(B, N, H, D, drop, rows, q8):
    ext = _ext.ext()
    assert ext.attn_bwd_bias_rows(B, N, H, D, drop) == rows
    assert ext.attn_bwd_q8_ok(B, N, H, D, drop) == q8
