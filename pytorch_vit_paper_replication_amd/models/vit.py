"""Vision Transformer (Dosovitskiy et al., 2020) with the reference's public surface.

API parity with the reference ``models/vit.py``:
  * ``ViT(image_size=224, patch_size=16, num_transformer_layer=12, num_heads=12, embedding_dim=768,
    mlp_size=3072, attn_dropout=0, mlp_dropout=0.1, embedding_dropout=0.1, num_classes=1000)``
    (reference models/vit.py:173-183) and ``forward(x [B,3,H,W]) -> logits [B, num_classes]``;
  * sub-blocks ``PatchEmbedding`` (:5-67), ``MultiHeadSelfAttentionBlock`` (:69-98),
    ``MLPBlock`` (:100-131), ``TransformerEncoderBlock`` (:133-169) with the same constructor
    signatures and submodule names, hence the same 152-key ``state_dict``;
  * the same initialisation, in the same RNG order (CLS/pos ``torch.rand``, Conv/Linear kaiming,
    in_proj xavier, zero MHA biases), so a seeded model is bit-identical to the reference's.

Execution: on CPU (or with ``PVR_DISABLE_FUSED=1``) every module runs plain PyTorch fp32 math
equivalent to the reference. On an MI355X the top-level ``ViT.forward`` runs the fused path: flat
parameter store with a bf16 shadow, hand-written gfx950 kernels for patch embedding, LayerNorm,
MFMA GEMMs with fused bias/GELU/dropout/residual epilogues, flash-style attention and a fused
classifier head (``ops.fused_vit``), with hand-written backward passes.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from .. import _ext


class PatchEmbedding(nn.Module):
    """Image -> [B, N+1, D] patch + CLS + position embeddings (reference models/vit.py:5-67)."""

    def __init__(self, image_size: int, color_channels: int = 3, patch_size: int = 16,
                 embedding_dropout: float = 0.1, embedding_dim: int = 768):
        super().__init__()
        self.patch_size = patch_size
        assert image_size % self.patch_size == 0, (
            f"Input image size must be divisible by patch size, image size: {image_size}, patch_size: {patch_size}")
        self.number_of_patches = int((image_size ** 2) / (patch_size ** 2))
        self.patch_and_flatten = nn.Sequential(
            nn.Conv2d(in_channels=color_channels, out_channels=embedding_dim, kernel_size=patch_size, stride=patch_size),
            nn.Flatten(start_dim=2, end_dim=3),
        )
        self.class_token = nn.Parameter(torch.rand(1, 1, embedding_dim), requires_grad=True)
        self.position_embedding = nn.Parameter(torch.rand(1, self.number_of_patches + 1, embedding_dim),
                                               requires_grad=True)
        self.dropout = nn.Dropout(p=embedding_dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b = x.shape[0]
        cls = self.class_token.expand(b, -1, -1)
        x = self.patch_and_flatten(x).permute(0, 2, 1)
        x = torch.cat((cls, x), dim=1) + self.position_embedding
        return self.dropout(x)


class SelfAttention(nn.Module):
    """Multi-head attention with ``nn.MultiheadAttention``'s parameter layout and init.

    Parameters ``in_proj_weight [3D, D]`` (rows q;k;v), ``in_proj_bias [3D]``, ``out_proj.{weight,bias}``,
    so checkpoints interchange with the reference's ``nn.MultiheadAttention(batch_first=True)``.
    """

    def __init__(self, embed_dim: int, num_heads: int, dropout: float = 0.0, batch_first: bool = True):
        super().__init__()
        assert embed_dim % num_heads == 0, "embed_dim must be divisible by num_heads"
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.dropout = dropout
        self.batch_first = batch_first
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        # created (and default-initialised) before in_proj, exactly like nn.MultiheadAttention
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=True)
        self._reset_parameters()

    def _reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.constant_(self.in_proj_bias, 0.0)
        nn.init.constant_(self.out_proj.bias, 0.0)

    def forward(self, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, need_weights: bool = False,
                attn_mask: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        if not self.batch_first:
            query, key, value = (t.transpose(0, 1) for t in (query, key, value))
        B, Nq, D = query.shape
        Nk = key.shape[1]
        H, dh = self.num_heads, self.head_dim
        w_q, w_k, w_v = self.in_proj_weight.chunk(3)
        b_q, b_k, b_v = self.in_proj_bias.chunk(3)
        if query is key and key is value:
            q, k, v = F.linear(query, self.in_proj_weight, self.in_proj_bias).chunk(3, dim=-1)
        else:
            q, k, v = F.linear(query, w_q, b_q), F.linear(key, w_k, b_k), F.linear(value, w_v, b_v)
        q = q.view(B, Nq, H, dh).transpose(1, 2)
        k = k.view(B, Nk, H, dh).transpose(1, 2)
        v = v.view(B, Nk, H, dh).transpose(1, 2)
        p = self.dropout if self.training else 0.0
        weights = None
        if need_weights:
            s = (q @ k.transpose(-2, -1)) / math.sqrt(dh)
            if attn_mask is not None:
                s = s + attn_mask
            a = torch.softmax(s, dim=-1)
            weights = a.mean(dim=1)
            a = F.dropout(a, p=p, training=p > 0)
            o = a @ v
        else:
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, dropout_p=p)
        o = o.transpose(1, 2).reshape(B, Nq, D)
        # a functional call on out_proj's parameters, as in nn.MultiheadAttention (so module hooks and
        # torchinfo-style accounting see this layer exactly as they see the reference's MHA)
        o = F.linear(o, self.out_proj.weight, self.out_proj.bias)
        if not self.batch_first:
            o = o.transpose(0, 1)
        return o, weights


class MultiHeadSelfAttentionBlock(nn.Module):
    """LN -> MSA (reference models/vit.py:69-98); the residual is added by the caller."""

    def __init__(self, embedding_dim: int = 768, num_heads: int = 12, attn_dropout: float = 0):
        super().__init__()
        self.layer_norm = nn.LayerNorm(normalized_shape=embedding_dim)
        self.multi_head_attention = SelfAttention(embed_dim=embedding_dim, num_heads=num_heads,
                                                  dropout=attn_dropout, batch_first=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        normalized_x = self.layer_norm(x)
        attn_output, _ = self.multi_head_attention(query=normalized_x, key=normalized_x, value=normalized_x,
                                                   need_weights=False)
        return attn_output


class MLPBlock(nn.Module):
    """LN -> Linear -> GELU -> Dropout -> Linear -> Dropout (reference models/vit.py:100-131)."""

    def __init__(self, embedding_dim: int = 768, mlp_size: int = 3072, dropout: float = 0.1):
        super().__init__()
        self.layer_norm = nn.LayerNorm(normalized_shape=embedding_dim)
        self.mlp = nn.Sequential(
            nn.Linear(in_features=embedding_dim, out_features=mlp_size),
            nn.GELU(),
            nn.Dropout(p=dropout),
            nn.Linear(in_features=mlp_size, out_features=embedding_dim),
            nn.Dropout(p=dropout),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.mlp(self.layer_norm(x))


class TransformerEncoderBlock(nn.Module):
    """x = MSA(x) + x ; x = MLP(x) + x (reference models/vit.py:133-169)."""

    def __init__(self, embedding_dim: int = 768, num_heads: int = 12, attn_dropout: float = 0,
                 mlp_size: int = 3072, mlp_dropout: float = 0.1):
        super().__init__()
        self.msa_block = MultiHeadSelfAttentionBlock(embedding_dim=embedding_dim, num_heads=num_heads,
                                                     attn_dropout=attn_dropout)
        self.mlp_block = MLPBlock(embedding_dim=embedding_dim, mlp_size=mlp_size, dropout=mlp_dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.msa_block(x) + x
        x = self.mlp_block(x) + x
        return x

    # fused-path helpers ---------------------------------------------------------------
    def fused_params(self):
        m, p = self.msa_block, self.mlp_block
        a = m.multi_head_attention
        return (m.layer_norm.weight, m.layer_norm.bias, a.in_proj_weight, a.in_proj_bias,
                a.out_proj.weight, a.out_proj.bias, p.layer_norm.weight, p.layer_norm.bias,
                p.mlp[0].weight, p.mlp[0].bias, p.mlp[3].weight, p.mlp[3].bias)


class ViT(nn.Module):
    """ViT-Base/16 by default (reference models/vit.py:172-236)."""

    def __init__(self, image_size: int = 224, patch_size: int = 16, num_transformer_layer: int = 12,
                 num_heads: int = 12, embedding_dim: int = 768, mlp_size: int = 3072, attn_dropout: float = 0,
                 mlp_dropout: float = 0.1, embedding_dropout: float = 0.1, num_classes: int = 1000):
        super().__init__()
        self.patch_embedding_block = PatchEmbedding(image_size=image_size, patch_size=patch_size,
                                                    embedding_dim=embedding_dim, embedding_dropout=embedding_dropout)
        self.transformer_encoder = nn.Sequential(*[
            TransformerEncoderBlock(embedding_dim=embedding_dim, num_heads=num_heads, attn_dropout=attn_dropout,
                                    mlp_size=mlp_size, mlp_dropout=mlp_dropout)
            for _ in range(num_transformer_layer)])
        self.layer_norm = nn.LayerNorm(normalized_shape=embedding_dim)
        self.classifier = nn.Sequential(nn.Linear(in_features=embedding_dim, out_features=num_classes))
        self.config = dict(image_size=image_size, patch_size=patch_size, num_transformer_layer=num_transformer_layer,
                           num_heads=num_heads, embedding_dim=embedding_dim, mlp_size=mlp_size,
                           attn_dropout=attn_dropout, mlp_dropout=mlp_dropout, embedding_dropout=embedding_dropout,
                           num_classes=num_classes)

    # ------------------------------------------------------------------ reference path
    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        x = self.patch_embedding_block(x)
        x = self.transformer_encoder(x)
        return self.layer_norm(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _ext.use_fused(x) and self._fused_supported(x):
            return self._forward_fused(x)
        x = self.forward_features(x)
        return self.classifier(x[:, 0])

    # ------------------------------------------------------------------ fused path
    def _fused_supported(self, x: torch.Tensor) -> bool:
        c = self.config
        D, H = c["embedding_dim"], c["num_heads"]
        if x.dim() != 4 or x.shape[1] != 3 or D % H != 0 or D // H not in (64, 80, 96, 128) or D % 64 != 0:
            return False
        if c["mlp_size"] % 64 != 0:
            return False
        P = c["patch_size"]
        return x.shape[2] == x.shape[3] == c["image_size"] and x.shape[2] % P == 0

    @staticmethod
    def _rank_offset() -> int:
        # per-rank offset of the dropout counter: DDP ranks draw different masks from one base
        dist = torch.distributed
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        return rank * 40503

    def _dropout_seed(self, device) -> torch.Tensor:
        rng = getattr(self, "_pvr_rng", None)
        if rng is not None and rng.device != device:
            with torch.inference_mode(False):  # e.g. restored on the CPU before .cuda(): keep the counter
                rng = rng.to(device)
            object.__setattr__(self, "_pvr_rng", rng)
        if rng is None:
            with torch.inference_mode(False):
                base = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
                rng = torch.tensor([base * 2654435761 + self._rank_offset()], dtype=torch.int64, device=device)
            object.__setattr__(self, "_pvr_rng", rng)
        seed = torch.empty_like(rng)
        _ext.ext().rng_next(rng, seed)  # seed = rng; rng += 1 (one device kernel, graph-replay safe)
        return seed

    def _forward_fused(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops.fused_vit import HeadFn

        tokens, store, B, N = self._fused_encoder(x)
        head = self.classifier[0]
        return HeadFn.apply(tokens, B, N, self.layer_norm.eps, store, self.layer_norm.weight, self.layer_norm.bias,
                            head.weight, head.bias)

    def _fused_encoder(self, x: torch.Tensor):
        """Patch embedding + every encoder block on the fused path: (bf16 tokens [B*N, D], store, B, N).
        Shared by this model's head and the classifier-free backbone (models/vit_no_classifier.py)."""
        from ..ops.fused_vit import ATTN_SITE, EncoderBlockFn, block_links, PatchEmbedFn, site_drop
        from ..runtime.param_store import get_store

        c = self.config
        dev = x.device
        for p in self.parameters():
            if p.device != dev:
                raise RuntimeError(f"input is on {dev} but model parameters are on {p.device}")
        store = get_store(self, dev)
        store.join_side()
        store.refresh_shadow()
        if not getattr(store, "_vit_t_registered", False):
            store.register_transposed([w for blk in self.transformer_encoder for w in blk.fused_params()[2:12:2] if w.dim() == 2])
            store._vit_t_registered = True
        store.ensure_transposed()
        training = self.training
        grad = torch.is_grad_enabled()
        store.grad_enabled = grad  # the fused Functions' forward runs with grad mode off: tell them
        if grad:
            store.prepare_grads()
        need_seed = training and (c["mlp_dropout"] > 0 or c["embedding_dropout"] > 0 or c["attn_dropout"] > 0)
        seed = self._dropout_seed(dev) if need_seed else None
        pe = self.patch_embedding_block
        conv = pe.patch_and_flatten[0]
        tokens = PatchEmbedFn.apply(x, c["patch_size"], store, seed, pe.dropout.p, training,
                                    conv.weight, conv.bias, pe.class_token, pe.position_embedding)
        B = x.shape[0]
        N = pe.number_of_patches + 1
        f8 = self._fp8_state(dev, B * N)
        if f8 is not None:
            f8.begin_step(training)
        blocks = list(self.transformer_encoder)
        drops2 = [site_drop(seed, 2 + 2 * i, blk.mlp_block.mlp[4].p, training) for i, blk in enumerate(blocks)]
        links = block_links(blocks, drops2)
        for i, blk in enumerate(blocks):
            ln1 = blk.msa_block.layer_norm
            ln2 = blk.mlp_block.layer_norm
            mha = blk.msa_block.multi_head_attention
            drops = (site_drop(seed, 1 + 2 * i, blk.mlp_block.mlp[2].p, training), drops2[i],
                     site_drop(seed, ATTN_SITE + i, mha.dropout, training))
            tokens = EncoderBlockFn.apply(tokens, B, N, mha.num_heads, ln1.eps, ln2.eps, store, drops,
                                          None if f8 is None else (f8, i), links[i], *blk.fused_params())
        return tokens, store, B, N

    # ------------------------------------------------------------------ fp8
    def enable_fp8(self, enabled: bool = True, history: int = 16, margin: int = 0, dgrad: bool = True,
                   wgrad: bool = True, grad_fmt: str = "e4m3") -> "ViT":
        """Run the encoder's GEMMs in fp8 on the fused MI355X path (ops/fp8.py), per-tensor delayed
        scaling with an amax history of ``history`` steps:

        * forward GEMMs: e4m3 activations x e4m3 weights;
        * ``dgrad=True`` (default): the backward's activation-gradient GEMMs too, e5m2 gradients x
          e4m3 transposed weights. This changes the backward numerics (``tests/kernel_checks.py``
          ``check_vit_fp8_dgrad`` pins the per-tensor error); ``dgrad=False`` keeps them bf16;
        * ``wgrad=True`` (default, with ``dgrad``): the weight-gradient GEMMs too, e5m2 gradients^T x
          e4m3 activations^T (transposed quantize passes with the same slots' scales) from the second
          step on (``check_vit_fp8_wgrad`` pins the per-tensor error, 1-8 % rel-L2 per weight
          gradient); ``wgrad=False`` keeps them bf16 (20 % of the ViT-H/14 fp8 throughput). Round 5
          made it opt-in on a 3-seed study that could not discriminate; round 6's 6-seed ViT-H/14 study
          (``profiles/r6/fp8_study/stats.md``, windowed training loss at steps 200 / 400 / 600 of a
          1000-step schedule, paired by seed) finds both fp8 variants within one bf16 standard
          deviation at every checkpoint and no significant paired difference (p 0.08-0.33), with the
          fp8 means 6-29 % above bf16's at steps 400 / 600: a trend more seeds would be needed to
          confirm or rule out;
        * ``grad_fmt``: the gradients' fp8 format in the dgrad / wgrad GEMMs, ``"e4m3"`` (default
          since round 6) or ``"e5m2"``. Round 6 measured the weight-gradient GEMM error on captured
          ViT-B/16 operands (``profiles/r6/mx_study``): the error comes from e5m2's 2-bit mantissa;
          per-32-element MX block scales change nothing. With e4m3 gradients (same per-tensor delayed
          scaling) the mean per-tensor error of all encoder gradients against the bf16 backward halves
          (0.036 vs 0.072, ``check_vit_fp8_grad_formats``), and in the 6-seed ViT-H/14 study
          (``profiles/r6/e4m3_study/stats.md``) the e4m3 run is closer to bf16 at every checkpoint (the
          one significant fp8 gap, e5m2 at step 400, p 0.008, is gone: p 0.135). The format is a
          runtime argument of every kernel that writes a gradient copy (the dgrad epilogues, LayerNorm
          backward, attention backward, column sums), so both formats run at the same speed;
        * attention, LayerNorm, the patch embedding / head GEMMs and the optimizer stay bf16 / fp32.

        The constructor signature stays the reference's; fp8 is opt-in."""
        old = getattr(self, "_fp8_cfg", None)
        if grad_fmt not in ("e5m2", "e4m3"):
            raise ValueError(f"enable_fp8: grad_fmt must be 'e5m2' or 'e4m3', got {grad_fmt!r}")
        cfg = (history, margin, bool(dgrad), bool(wgrad), grad_fmt) if enabled else None
        object.__setattr__(self, "_fp8_cfg", cfg)
        if cfg is None or old is None or old[:2] != cfg[:2] or old[4:] != cfg[4:]:
            object.__setattr__(self, "_fp8", None)  # new scaling state; only a dgrad switch keeps the histories
        return self

    def _fp8_state(self, device, tokens: int):
        cfg = getattr(self, "_fp8_cfg", None)
        if cfg is None:
            return None
        from ..ops import fp8 as F8

        c = self.config
        if not F8.supported(tokens, c["embedding_dim"], c["mlp_size"]):
            return None
        st = getattr(self, "_fp8", None)
        if st is None or st.device != device:
            old_sd = st.state_dict() if st is not None else getattr(self, "_fp8_pending", None)
            st = F8.Fp8State(c["num_transformer_layer"], device, history=cfg[0], margin=cfg[1], dgrad=cfg[2], wgrad=cfg[3],
                             grad_fmt=F8.E4M3 if cfg[4] == "e4m3" else F8.E5M2)
            if old_sd is not None:  # restored (or built) on another device: carry the scaling state over
                st.load_state_dict(old_sd)
            object.__setattr__(self, "_fp8", st)
            object.__setattr__(self, "_fp8_pending", None)
        st.dgrad = cfg[2]
        st.wgrad = cfg[3] and cfg[2]
        return st

    # ------------------------------------------------------------------ resume state
    def runtime_state_dict(self) -> dict:
        """Fused-path state outside ``state_dict()`` that a bit-exact resume needs (CPU tensors, loads
        with ``weights_only=True``): the device dropout counter (next seed of the counter-based masks)
        and the fp8 delayed-scaling state (amax histories, scales, calibration flags)."""
        out = {}
        rng = getattr(self, "_pvr_rng", None)
        if rng is not None:
            # rank-free: every DDP rank re-adds its own offset on load (rank 0 writes the checkpoint)
            out["dropout_rng"] = rng.detach().cpu().clone() - self._rank_offset()
            out["dropout_rng_rank_free"] = torch.ones(1, dtype=torch.int64)
        st = getattr(self, "_fp8", None)
        if st is not None:
            out["fp8"] = st.state_dict()
        return out

    def load_runtime_state_dict(self, sd: dict, device=None) -> None:
        """Restore :meth:`runtime_state_dict` (``device``: where the fused path will run; default the
        parameters' device). The fp8 state needs ``enable_fp8`` with the same history first."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        if "dropout_rng" in sd:
            rng = sd["dropout_rng"].to(dtype=torch.int64).clone()
            if "dropout_rng_rank_free" in sd:
                rng += self._rank_offset()
            object.__setattr__(self, "_pvr_rng", rng.to(dev))  # moved to the forward's device on first use
        if "fp8" in sd:
            cfg = getattr(self, "_fp8_cfg", None)
            if cfg is None:
                raise RuntimeError("checkpoint holds fp8 scaling state: call enable_fp8(...) before loading it")
            if dev.type != "cuda":
                # the fused path builds its fp8 state on the forward's device: apply it there
                object.__setattr__(self, "_fp8", None)
                object.__setattr__(self, "_fp8_pending", sd["fp8"])
                return
            from ..ops import fp8 as F8

            st = getattr(self, "_fp8", None)
            if st is None or st.device != dev:
                st = F8.Fp8State(self.config["num_transformer_layer"], dev, history=cfg[0], margin=cfg[1],
                                 dgrad=cfg[2], wgrad=cfg[3], grad_fmt=F8.E4M3 if cfg[4] == "e4m3" else F8.E5M2)
                object.__setattr__(self, "_fp8", st)
            st.load_state_dict(sd["fp8"])

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())
