"""Loader for the in-tree gfx950 extension ``_C`` (built by :mod:`.build`).

Policy: on a GPU tensor the fused HIP path is mandatory. If the extension cannot be loaded while a
GPU is present, :func:`use_fused` raises instead of silently running PyTorch fallbacks — set
``PVR_ALLOW_TORCH_FALLBACK=1`` to opt into the plain-PyTorch path on purpose (that is how the
reference-style baseline is benchmarked). On CPU the PyTorch reference path always runs.
"""
from __future__ import annotations

import contextlib
import os

import torch

_C = None
_ERR: BaseException | None = None
_TRIED = False


class StaleExtensionError(RuntimeError):
    """The in-tree ``_C`` was built from other ``csrc/`` sources than the ones in the tree."""


def check_source_hash(so, csrc) -> str:
    """Compare the source hash compiled into ``so`` with the hash of the sources in ``csrc``;
    returns the hash, raises :class:`StaleExtensionError` on a mismatch (or a binary without one)."""
    from .build import embedded_hash, source_hash

    want = source_hash(csrc)
    have = embedded_hash(so)
    if have != want:
        raise StaleExtensionError(
            f"{so} was built from other sources (binary {have}, csrc/ {want}): rebuild with "
            "`python -m pytorch_vit_paper_replication_amd.build` (or set PVR_AUTOBUILD=1)")
    return want


def load():
    """Import the compiled extension once; returns the module or None.

    The binary must carry the content hash of the ``csrc/`` sources next to it (build.py compiles
    it in): a stale ``_C`` is rebuilt first under ``PVR_AUTOBUILD=1`` and refused otherwise, so an
    edited kernel can never be tested through an old binary."""
    global _C, _ERR, _TRIED
    if _TRIED:
        return _C
    _TRIED = True
    debug = os.environ.get("PVR_DEBUG_KERNELS", "0") == "1"
    try:
        from .build import CSRC, ext_path

        if CSRC.is_dir() and ext_path(debug).exists():
            try:
                check_source_hash(ext_path(debug), CSRC)
            except StaleExtensionError:
                if os.environ.get("PVR_AUTOBUILD", "0") != "1":
                    raise
                from .build import build_extension

                build_extension(debug=debug)
                check_source_hash(ext_path(debug), CSRC)
        if debug:  # kernels with device-side invariant checks (build_extension(debug=True))
            from . import _C_debug as mod  # noqa: F401
        else:
            from . import _C as mod  # noqa: F401  (built in-tree)

        _C = mod
    except BaseException as e:  # pragma: no cover - depends on build state
        _ERR = e
        if os.environ.get("PVR_AUTOBUILD", "0") == "1":
            try:
                from .build import build_extension

                build_extension(debug=debug)
                if debug:
                    from . import _C_debug as mod2
                else:
                    from . import _C as mod2

                _C = mod2
                _ERR = None
            except BaseException as e2:
                _ERR = e2
    return _C


def available() -> bool:
    return load() is not None


_DETERMINISTIC_ENV = os.environ.get("PVR_DETERMINISTIC", "0") not in ("", "0")


def deterministic() -> bool:
    """Deterministic reductions on the fused path (``set_deterministic`` / ``PVR_DETERMINISTIC=1`` /
    ``torch.use_deterministic_algorithms(True)``): every bias / LayerNorm-parameter gradient and the
    weight gradients are reduced in a fixed order, so a training step produces the same bits on every
    run. Off by default: the float-atomic reductions are order-dependent in the last bits.

    The attention backward at sequence lengths with several 256-key blocks that take neither its
    last-key nor its tail-split slab path (e.g. N = 400, 677) sums dQ with float atomics by default;
    in deterministic mode each key block stores an f32 dQ slab and one pass sums the slabs in key-block
    order (``dq_slab_sum_kernel``; ``tests/kernel_checks.py::check_attn_bwd_det``).

    Each fused backward entry point calls this, so the native flag follows
    ``torch.use_deterministic_algorithms`` from the first backward kernel of a step on."""
    m = _C if _TRIED else load()
    on = torch.are_deterministic_algorithms_enabled() or _DETERMINISTIC_ENV
    if m is not None and bool(m.deterministic()) != on:
        m.set_deterministic(on)
    return on


@contextlib.contextmanager
def deterministic_mode(on: bool = True):
    """Context: deterministic reductions inside the block (see :func:`deterministic`)."""
    global _DETERMINISTIC_ENV
    old = _DETERMINISTIC_ENV
    _DETERMINISTIC_ENV = on
    try:
        deterministic()
        yield
    finally:
        _DETERMINISTIC_ENV = old
        deterministic()


def ext():
    m = load()
    if m is None:
        raise RuntimeError(
            "pytorch_vit_paper_replication_amd: the gfx950 extension _C is not built or failed to load "
            f"({_ERR!r}). Build it with `python -m pytorch_vit_paper_replication_amd.build`."
        )
    return m


def fallback_allowed() -> bool:
    return os.environ.get("PVR_ALLOW_TORCH_FALLBACK", "0") == "1"


_FORCE_REFERENCE = 0


def fused_disabled() -> bool:
    return _FORCE_REFERENCE > 0 or os.environ.get("PVR_DISABLE_FUSED", "0") == "1"


@contextlib.contextmanager
def reference_path():
    """Run the module-by-module PyTorch path inside the block, even on the GPU (used by
    :func:`utils.summary.summary`, whose per-module hooks the fused encoder would bypass)."""
    global _FORCE_REFERENCE
    _FORCE_REFERENCE += 1
    try:
        yield
    finally:
        _FORCE_REFERENCE -= 1


def use_fused(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the HIP kernels should run on it."""
    if not t.is_cuda:
        return False
    if fused_disabled():
        return False
    if available():
        return True
    if fallback_allowed():
        return False
    ext()  # raises with the load error
    return False


def free_scratch() -> None:
    """Return the extension's per-(device, stream) scratch buffers to the caching allocator: the
    split-K GEMM workspaces and tail slabs, the deterministic-mode partial rows, the attention
    backward's dQ accumulator and scratch (up to ~0.9 GB per layer size at ViT-L/16 384 px). Waits
    for the device first; the next fused call re-creates what it needs. Call it before
    ``torch.cuda.empty_cache()`` when switching model sizes in one process."""
    m = _C if _TRIED else load()
    if m is None:
        return
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    m.free_scratch()
    from .ops import gemm as _gemm

    _gemm._workspaces.clear()
