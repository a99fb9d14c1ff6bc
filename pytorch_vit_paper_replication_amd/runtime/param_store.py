"""Flat parameter / gradient / bf16-shadow store for the fused GPU path.

On the first fused forward on a device, every parameter of the model is re-pointed (``p.data``)
into one contiguous fp32 master buffer, and ``p.grad`` into one contiguous fp32 gradient buffer
(the same Parameter objects survive, so an optimizer built before ``model.to(device)`` keeps
working — SURVEY.md §3.4). A bf16 shadow of the master buffer feeds the MFMA GEMMs; it is
refreshed by one cast kernel whenever a parameter changed outside the fused optimizer (detected
from the per-parameter autograd version counters), and written directly by
:class:`~pytorch_vit_paper_replication_amd.optim.FusedAdam` otherwise.

The fused autograd Functions write weight gradients straight into the gradient views (split-K
wgrad GEMMs accumulate with f32 atomics, bias/LN gradients are reduced in-kernel), so the
gradient buffer doubles as the data-parallel all-reduce buckets (``parallel.ddp``): no copy into
bucket storage and no per-tensor collectives. ``grad_ready`` notifies listeners (the DDP
bucketer) as soon as a group of parameters has its final gradient.
"""
from __future__ import annotations

import weakref
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

import torch

from .. import _ext

ALIGN = 64  # elements; keeps every parameter 256-B aligned and 4-element vectorisable
# weight-gradient GEMMs on a second stream (module attribute, not an env knob: the side-stream
# ordering test switches it off to compare against the serial schedule)
SIDE_WGRAD = True
# Bytes of side-stream weight-gradient inputs held at once (0: every batch until the end-of-backward
# join). Once more is held, the oldest batches are released: the stream that produced their tensors
# first waits for that batch's completion event, so the blocks are reused in stream order. Each such
# wait can stall the dgrad chain behind the low-priority side stream, so the bound is in bytes and
# generous: ViT-B/16 b256 holds ~1 GB and never waits (a 4-batch window there cost 1.2 % per step),
# ViT-H/14 fp8 b256 peaked at 158.5 GB unbounded vs 133 GB with a 4-batch window (ADVICE r3,
# profiles/r4/side_window.md).
SIDE_HOLD_BYTES = 16 << 30
SIDE_WINDOW = 0  # alternatively a batch-count bound (A/B)


def _norm_device(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def unique_params(module: torch.nn.Module):
    """(names, parameters) in registration order, shared parameters once: the store's layout order."""
    seen = set()
    params: List[torch.nn.Parameter] = []
    names: List[str] = []
    for n, p in module.named_parameters():
        if id(p) in seen:
            continue
        seen.add(id(p))
        params.append(p)
        names.append(n)
    return names, params


class ParamStore:
    """``layout = (starts, align)`` (optional): the parameters with these indices begin at a multiple
    of ``align`` elements and the buffers end at one — the data-parallel bucketer passes its buckets'
    first parameters, so every bucket is a whole number of ``align``-element blocks (zero padding
    between buckets; it stays zero through backward, the all-reduce and the optimizer)."""

    def __init__(self, module: torch.nn.Module, device: torch.device, layout=None):
        names, params = unique_params(module)
        self.device = _norm_device(device)
        self.layout = layout
        # grad mode at the model call, set by the model's fused forward: the autograd Functions' own
        # forward always runs with grad mode off, so an inference call is told here (no saved tensors)
        self.grad_enabled = True
        self.params = params
        self.names = names
        self.offsets: List[int] = []
        starts, big = (layout if layout is not None else ((), ALIGN))
        starts = set(starts)
        off = 0
        for i, p in enumerate(params):
            if i in starts:
                off = (off + big - 1) // big * big
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        if starts:
            off = (off + big - 1) // big * big
        self.numel = max(off, ALIGN)
        self._index: Dict[int, int] = {id(p): i for i, p in enumerate(params)}
        with torch.inference_mode(False), torch.no_grad():
            self.flat = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self.grad_flat = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self.shadow = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            self._views = []
            self._gviews = []
            self._sviews = []
            for p, o in zip(params, self.offsets):
                n = p.numel()
                v = self.flat[o:o + n].view(p.shape)
                v.copy_(p.data.to(self.device, torch.float32).reshape(p.shape))
                old_grad = p.grad
                p.data = v
                gv = self.grad_flat[o:o + n].view(p.shape)
                if old_grad is not None:
                    gv.copy_(old_grad.to(self.device, torch.float32).reshape(p.shape))
                self._views.append(v)
                self._gviews.append(gv)
                self._sviews.append(self.shadow[o:o + n].view(p.shape))
                if p.requires_grad:
                    p.grad = gv
                p._pvr_store_ref = weakref.ref(self)
        self._shadow_key: Optional[int] = None
        self._t_params: List[torch.nn.Parameter] = []
        self._t_views: Dict[int, torch.Tensor] = {}
        self._t_meta: Optional[torch.Tensor] = None
        self._t_tiles = 0
        self._t_dirty = True
        self.shadow_t: Optional[torch.Tensor] = None
        self._listeners: List[Callable[[List[torch.nn.Parameter]], None]] = []
        self.generation = 0  # bumped whenever the bf16 shadow changes (derived caches key on it)
        # weight-gradient side stream (see on_side): created lazily on GPU stores
        self._side: Optional[torch.cuda.Stream] = None
        self._side_pending = False
        self._join_queued = False
        # (producing stream, held tensors, side-stream completion event) per queued batch
        self._side_refs: List[Tuple[torch.cuda.Stream, Tuple[torch.Tensor, ...], Any, int]] = []
        self._side_bytes = 0
        self.refresh_shadow(force=True)

    # ------------------------------------------------------------------ validity
    def covers(self, module: torch.nn.Module) -> bool:
        """True if every parameter of ``module`` still lives in this store's buffers."""
        for p in module.parameters():
            i = self._index.get(id(p))
            if i is None or p.data.data_ptr() != self._views[i].data_ptr() or p.device != self.device:
                return False
        return True

    def covers_param(self, p: torch.nn.Parameter) -> bool:
        i = self._index.get(id(p))
        return i is not None and p.device == self.device and p.data.data_ptr() == self._views[i].data_ptr()

    # ------------------------------------------------------------------ shadow
    def _version_key(self) -> int:
        return sum(p._version for p in self.params)

    def refresh_shadow(self, force: bool = False) -> None:
        key = self._version_key()
        if force or key != self._shadow_key:
            with torch.inference_mode(False), torch.no_grad():
                if self.flat.is_cuda and _ext.available():
                    _ext.ext().cast_f32_bf16(self.flat, self.shadow)
                else:
                    self.shadow.copy_(self.flat)
            self._shadow_key = key
            self._t_dirty = True
            self.generation += 1

    def mark_shadow_fresh(self, transposed: bool = False) -> None:
        """Called by the fused optimizer after it rewrote master + shadow in one pass (and, with
        ``transposed``, the W^T shadow of every registered weight too)."""
        self._shadow_key = self._version_key()
        if not transposed:
            self._t_dirty = True
        self.generation += 1

    def transposed_layout(self):
        """(registered weights, [flat offset, shadow_t offset, R, C, first 64x64 tile] rows) of the
        W^T shadow, or None when a weight's shape is not a multiple of 64 (then only the separate
        transpose pass handles it). Clean (not dirty) W^T is required by the optimizer's fused write."""
        if not self._t_params or self._t_meta is None:
            return None
        if any(p.shape[0] % 64 or p.shape[1] % 64 for p in self._t_params):
            return None
        return self._t_params, self._t_meta

    # ------------------------------------------------------------------ transposed bf16 weights
    def register_transposed(self, params: Iterable[torch.nn.Parameter]) -> None:
        """Keep a bf16 W^T copy of these 2-D weights (the dgrad GEMM's B operand, k-contiguous)."""
        ps = [p for p in params if id(p) not in self._t_views and p.dim() == 2]
        if not ps:
            return
        self._t_params.extend(ps)
        total = sum((p.numel() + ALIGN - 1) // ALIGN * ALIGN for p in self._t_params)
        with torch.inference_mode(False), torch.no_grad():
            self.shadow_t = torch.empty(total, dtype=torch.bfloat16, device=self.device)
            meta, off, tiles = [], 0, 0
            self._t_views = {}
            for p in self._t_params:
                R, C = p.shape
                self._t_views[id(p)] = self.shadow_t[off:off + p.numel()].view(C, R)
                meta.append([self.offset(p), off, R, C, tiles])
                tiles += ((R + 63) // 64) * ((C + 63) // 64)
                off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
            self._t_meta = torch.tensor(meta, dtype=torch.int64, device=self.device)
            self._t_tiles = tiles
        self._t_dirty = True

    def ensure_transposed(self) -> None:
        if not self._t_params or not self._t_dirty:
            return
        with torch.inference_mode(False), torch.no_grad():
            if self.flat.is_cuda and _ext.available():
                _ext.ext().transpose_batched(self.shadow, self.shadow_t, self._t_meta, self._t_tiles)
            else:
                for p in self._t_params:
                    self._t_views[id(p)].copy_(self.bf16(p).t())
        self._t_dirty = False

    def layout_key(self):
        """Identity of the bf16 shadow buffers (changes when register_transposed reallocates)."""
        return (self.shadow.data_ptr(), self.shadow_t.data_ptr() if self.shadow_t is not None else 0)

    def bf16_t(self, p: torch.nn.Parameter) -> Optional[torch.Tensor]:
        return self._t_views.get(id(p))

    def bf16(self, p: torch.nn.Parameter) -> torch.Tensor:
        return self._sviews[self._index[id(p)]]

    def offset(self, p: torch.nn.Parameter) -> int:
        return self.offsets[self._index[id(p)]]

    def contains(self, p: torch.nn.Parameter) -> bool:
        return id(p) in self._index

    # ------------------------------------------------------------------ gradients
    def prepare_grads(self) -> None:
        self.join_side()
        self._prepare_grads()

    def _prepare_grads(self) -> None:
        """Make every trainable parameter's .grad a view of the flat gradient buffer.

        ``zero_grad(set_to_none=True)`` leaves ``p.grad is None``, which means "zero": the region is
        cleared and the view re-attached. A foreign tensor a user assigned is copied in.
        """
        with torch.inference_mode(False), torch.no_grad():
            for i, p in enumerate(self.params):
                if not p.requires_grad:
                    continue
                gv = self._gviews[i]
                g = p.grad
                if g is None:
                    gv.zero_()
                    p.grad = gv
                elif g.data_ptr() != gv.data_ptr():
                    gv.copy_(g)
                    p.grad = gv

    def grad_dest(self, p: torch.nn.Parameter) -> Optional[torch.Tensor]:
        """fp32 gradient view to accumulate into, or None if the parameter is frozen."""
        if not p.requires_grad:
            return None
        i = self._index[id(p)]
        gv = self._gviews[i]
        g = p.grad
        if g is None:
            gv.zero_()
            p.grad = gv
        elif g.data_ptr() != gv.data_ptr():
            gv.copy_(g)
            p.grad = gv
        return gv

    def adopt_grad(self, p: torch.nn.Parameter) -> None:
        """Move a gradient autograd allocated outside the flat buffer into its view (DDP hook path)."""
        i = self._index.get(id(p))
        if i is None or p.grad is None:
            return
        gv = self._gviews[i]
        if p.grad.data_ptr() != gv.data_ptr():
            with torch.no_grad():
                gv.copy_(p.grad)
            p.grad = gv

    # ------------------------------------------------------------------ weight-gradient side stream
    # The weight-gradient GEMMs of a backward pass are off the critical path (only the optimizer and
    # the gradient all-reduce consume them), so the fused backward queues them on a second HIP stream:
    # they fill the CUs the dgrad chain leaves idle (last-round tile quantisation of N = 768 GEMMs,
    # memory-bound LayerNorm / attention phases). Ordering: the side stream waits for the main stream
    # before each batch of wgrads; gradient-ready notifications (DDP buckets) are issued from the side
    # stream after it has caught up with main; an end-of-backward autograd callback joins the side
    # stream back into the caller's stream, so anything after backward() sees complete gradients.
    def side_stream(self) -> Optional[torch.cuda.Stream]:
        if self.device.type != "cuda" or not SIDE_WGRAD:
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def on_side(self, fn: Callable[[], None], *tensors: torch.Tensor) -> None:
        """Run ``fn`` (kernel launches) on the side stream after the work queued so far on the
        current stream. ``tensors`` (produced on the current stream) are held until ``join_side``
        has made that stream wait for the side stream, and only then released: the caching allocator
        then reuses their blocks in stream order, as in a one-stream program. (``record_stream`` would
        instead keep each block out of reuse until the GPU has passed the side-stream work, so every
        step the host runs ahead of the GPU would hold a whole step of activations: at ViT-L/16 384 px
        batch 128 that exhausted the 288 GB and the allocator's free-and-retry stalled steps for
        seconds.) At most ``SIDE_HOLD_BYTES`` (or ``SIDE_WINDOW`` batches) are held at once: queueing
        more releases the oldest after its producer stream has waited for that batch's completion
        event."""
        side = self.side_stream()
        if side is None:
            fn()
            return
        from ..ops import gemm as _gemm  # (ops imports the runtime: resolved at call time)

        main = torch.cuda.current_stream(self.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            prev, _gemm.OVERLAPPED = _gemm.OVERLAPPED, True  # split widths for work beside the main stream
            try:
                fn()
            finally:
                _gemm.OVERLAPPED = prev
        done = None
        if SIDE_WINDOW > 0 or SIDE_HOLD_BYTES > 0:
            done = torch.cuda.Event()
            done.record(side)
        nbytes = sum(t.untyped_storage().nbytes() for t in tensors if isinstance(t, torch.Tensor))
        self._side_refs.append((main, tensors, done, nbytes))
        self._side_bytes += nbytes
        self._side_pending = True
        while len(self._side_refs) > 1 and ((SIDE_WINDOW > 0 and len(self._side_refs) > SIDE_WINDOW) or
                                            (SIDE_HOLD_BYTES > 0 and self._side_bytes > SIDE_HOLD_BYTES)):
            # release the oldest batch's inputs: their producer waits for the batch's wgrads first
            st, _, ev, nb = self._side_refs.pop(0)
            st.wait_event(ev)
            self._side_bytes -= nb
        self._queue_join()

    def _queue_join(self) -> None:
        if self._join_queued:
            return
        try:
            torch.autograd.Variable._execution_engine.queue_callback(self.join_side)
            self._join_queued = True
        except RuntimeError:  # not inside a backward pass: join eagerly
            self.join_side()

    def join_side(self) -> None:
        """Make the current stream (and every stream that produced a held tensor) wait for every
        side-stream launch so far, then release the held tensors."""
        self._join_queued = False
        if self._side_pending and self._side is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self._side)
            for s in {r[0] for r in self._side_refs}:
                if s != cur:
                    s.wait_stream(self._side)
            self._side_refs.clear()
            self._side_bytes = 0
            self._side_pending = False

    def zero_grad(self) -> None:
        self.join_side()
        g = self.grad_flat
        if g.is_cuda and _ext.available() and g.numel() % 4 == 0:
            _ext.ext().zero_f32(g)  # one 16-B-store kernel over the whole flat buffer
        else:
            g.zero_()
        for i, p in enumerate(self.params):
            if p.requires_grad:
                p.grad = self._gviews[i]

    def add_listener(self, fn: Callable[[List[torch.nn.Parameter]], None]) -> None:
        self._listeners.append(fn)

    def remove_listener(self, fn) -> None:
        if fn in self._listeners:
            self._listeners.remove(fn)

    def grad_ready(self, params: Iterable[torch.nn.Parameter]) -> None:
        if self._listeners:
            ps = [p for p in params if p is not None]
            if self._side_pending and self._side is not None:
                # gradients of this batch live on both streams: notify from the side stream once it
                # has caught up with main, so a collective gated on the current stream sees all of them
                self._queue_join()  # keep the join callback ahead of any listener's own callback
                self._side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(self._side):
                    for fn in self._listeners:
                        fn(ps)
                return
            for fn in self._listeners:
                fn(ps)


def lookup_store(p: torch.nn.Parameter) -> Optional[ParamStore]:
    """The live store that owns ``p`` (None if the parameter moved out of it)."""
    r = getattr(p, "_pvr_store_ref", None)
    st = r() if r is not None else None
    if st is None or not st.covers_param(p):
        return None
    return st


def get_store(module: torch.nn.Module, device: torch.device, layout=None) -> ParamStore:
    """Return the module's store for ``device``, (re)building it if parameters moved or (when
    ``layout`` is given) if its bucket layout differs. A rebuilt store copies values and gradients
    from the old one (the parameters still point into it); FusedAdam re-keys its state on it."""
    st: Optional[ParamStore] = getattr(module, "_pvr_store", None)
    if st is not None and st.device == _norm_device(device) and st.covers(module) and \
            (layout is None or st.layout == layout):
        return st
    if st is not None:
        st.join_side()
    st = ParamStore(module, device, layout)
    object.__setattr__(module, "_pvr_store", st)
    return st
