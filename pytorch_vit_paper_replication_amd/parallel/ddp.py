"""Data parallelism over RCCL/xGMI with gradient buckets overlapped with backward.

Design, MI355X-first rather than a copy of torch DDP:
  * the model's parameters live in one flat fp32 ``ParamStore``; its gradient buffer IS the bucket
    storage — buckets are contiguous slices, so there is no flatten/unflatten copy and every
    collective is one large message (xGMI links are point-to-point: few, big transfers);
  * parameters are broadcast from rank 0 with ONE collective over the flat master buffer (C1);
  * buckets are formed in reverse registration order (= backward order, last encoder block first),
    ``bucket_cap_mb`` each (default ≈ one ViT-B encoder block: 28 MB of fp32 gradients), except that
    the first-registered parameters (the embedding, whose gradients come last) form a final bucket of
    at most 4 MB: the first block's bucket then overlaps the embedding backward;
  * the fused backward Functions (or autograd hooks on the PyTorch path) report parameters as final;
    a full bucket is all-reduced immediately with ``async_op=True`` — RCCL runs it on its own stream
    ordered after the gradient kernels already queued, so it overlaps the remaining backward;
  * buckets launch strictly in index order on every rank (no collective-order mismatch), and an
    autograd end-of-backward callback flushes the rest and joins the stream before the optimizer
    (the global-norm clip therefore sees averaged gradients, C3).

Transport: each bucket is all-reduced with ``torch.distributed`` (ProcessGroupNCCL = RCCL on ROCm,
its own HIP stream, ``ReduceOp.AVG``), joined into the compute stream by ``work.wait()`` — no host
synchronisation; gloo / CPU the same way with a SUM + divide. World-1 A/B at ViT-B/16 b512
(profiles/r3/ddp_transport_world1_b512.log): no DDP 8082 / 8075 img/s, torch 8053, torch with the bf16
wire 8034 — RCCL's one-rank kernel (``oneRankReduce``, ~0.2 ms per bucket) hides under the backward.
(A framework-owned C++ RCCL communicator with its own mesh reduce-scatter schedule existed through
round 3; it was 8 % slower than this transport at world 1 with no identified cause, never used by
default, and was removed in round 4: ``comm`` accepts "auto" / "torch" only.)

Wire format (``comm_dtype``): fp32 by default. ``torch.bfloat16`` keeps a persistent bf16 mirror of
the gradient buffer (no per-step allocation): each bucket is cast into its slice, all-reduced in
bf16 (half the bytes on xGMI) and cast back. At 8 GPUs the fp32 gradients of ViT-B/16 (330 MB per
step) need ~2 ms of ring time against a ~60 ms backward at 512 images per GPU, fully hidden, so the
bf16 wire buys no step time there and costs two cast passes plus bf16 rounding of every gradient
(rel-L2 < 1e-2, tests/test_ddp_cpu.py): it is opt-in, for bandwidth-bound (multi-node, small-batch)
runs.

Bucket padding (``pad_buckets``, default on): every bucket is a whole number of world x 7 x 4 KiB
blocks — the flat store lays the buckets out on those boundaries with zero padding,
so a reduce-scatter splits each bucket into equal per-rank chunks of whole 4 KiB pages per xGMI link.
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn

from ..runtime.param_store import ParamStore, get_store, unique_params


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 28.0,
                 broadcast_parameters: bool = True, comm_dtype: Optional[torch.dtype] = None, comm: str = "auto",
                 timing: bool = False, pad_buckets: bool = True):
        super().__init__()
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("DistributedDataParallel needs an initialised torch.distributed process group")
        self.module = module
        self.process_group = process_group
        self.world = dist.get_world_size(process_group)
        self.bucket_cap = int(bucket_cap_mb * (1 << 20))
        self.broadcast_parameters = broadcast_parameters
        self.comm_dtype = comm_dtype
        self.pad_buckets = pad_buckets
        self.require_backward_grad_sync = True
        self._store: Optional[ParamStore] = None
        self._buckets: List[tuple] = []          # (start, end, [param indices])
        self._bucket_of: Dict[int, int] = {}
        self._pending: List[int] = []
        self._ready_ids = set()
        self._next_launch = 0
        self._works: List = []
        self._callback_queued = False
        self._hooks = []
        self._avg = dist.get_backend(process_group) == "nccl"
        if comm not in ("auto", "torch"):
            raise ValueError(f"DistributedDataParallel: unknown transport {comm!r} (torch.distributed only: 'auto' / 'torch')")
        self._comm_buf: Optional[torch.Tensor] = None  # persistent low-precision gradient mirror
        # per-bucket all-reduce timing (utils.metrics.StepLogger): (bytes, start, end) per launched
        # bucket, start = bucket ready on the compute stream, end = collective complete (HIP events
        # on GPU, host clock with gloo)
        self.timing = timing
        self._timings: List[tuple] = []
        self._timing_stream: Optional[torch.cuda.Stream] = None

    # ------------------------------------------------------------------ setup
    def _plan(self, params) -> List[List[int]]:
        """Bucket membership (parameter indices in launch order) from the parameters' order and sizes.

        The parameters registered first (ViT: class token, position embedding, patch conv) receive
        their gradients LAST, after the whole encoder backward: they get a small bucket of their own
        (<= 4 MB), so the bucket before it (the first encoder block) is all-reduced while the
        embedding backward still runs and only a few MB of collective remain after backward. The
        rest: reverse parameter order, contiguous flat ranges of about bucket_cap bytes."""
        tail_cap = min(self.bucket_cap, 4 << 20)
        tail: List[int] = []
        tail_bytes = 0
        for i in range(len(params)):
            nb = params[i].numel() * 4
            if tail and tail_bytes + nb > tail_cap:
                break
            tail.append(i)
            tail_bytes += nb
        buckets = []
        cur: List[int] = []
        cur_bytes = 0
        for i in reversed(range(len(tail), len(params))):
            cur.append(i)
            cur_bytes += params[i].numel() * 4
            if cur_bytes >= self.bucket_cap:
                buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            buckets.append(cur)
        if tail:
            buckets.append(list(reversed(tail)))
        return buckets

    def pad_elems(self) -> int:
        """Bucket granularity in fp32 elements: world x 7 x 4 KiB, so a ring or mesh
        reduce-scatter splits every bucket into equal per-rank chunks of whole 4 KiB pages per xGMI
        link (7 links per MI355X). 0 = unpadded (``pad_buckets=False``)."""
        return self.world * 7 * 1024 if self.pad_buckets else 0

    # ------------------------------------------------------------------ setup
    def _setup(self, device):
        st = getattr(self.module, "_pvr_store", None)
        if st is not None and st is self._store and st.covers(self.module):
            return st
        _, params = unique_params(self.module)
        plan = self._plan(params)
        pad = self.pad_elems()
        layout = (tuple(sorted(min(idxs) for idxs in plan)), pad) if pad else None
        store = get_store(self.module, device, layout=layout)
        if store is self._store:
            return store
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._store is not None:
            self._store.remove_listener(self._on_ready)
        self._store = store
        if self.broadcast_parameters:
            with torch.no_grad():
                src = dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0
                dist.broadcast(store.flat, src=src, group=self.process_group)
                for b in self.module.buffers():
                    dist.broadcast(b, src=src, group=self.process_group)
            store.refresh_shadow(force=True)
        if self.comm_dtype is not None and self.comm_dtype != store.grad_flat.dtype:
            self._comm_buf = torch.empty(store.numel, dtype=self.comm_dtype, device=store.grad_flat.device)
        self._buckets = []
        self._bucket_of = {}
        for bi, idxs in enumerate(plan):
            lo = min(store.offsets[i] for i in idxs)
            hi_i = max(idxs)
            hi = store.offsets[hi_i + 1] if hi_i + 1 < len(store.params) else store.numel
            self._buckets.append((lo, hi, idxs))
            for i in idxs:
                self._bucket_of[id(store.params[i])] = bi
        store.add_listener(self._on_ready)
        for p in store.params:
            if p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._autograd_hook))
        return store

    def _reset(self):
        st = self._store
        self._pending = [sum(1 for i in idxs if st.params[i].requires_grad) for (_, _, idxs) in self._buckets]
        self._ready_ids = set()
        self._next_launch = 0
        self._works = []
        self._timings = []  # one step's bucket timings (a step nobody popped is dropped here)
        self._callback_queued = False

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        dev = next(self.module.parameters()).device
        store = self._setup(dev)
        if torch.is_grad_enabled():
            store.prepare_grads()
        self._reset()
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    # ------------------------------------------------------------------ backward hooks
    def _autograd_hook(self, p):
        # PyTorch-path gradient: if autograd allocated it (zero_grad(set_to_none) after forward, as the
        # reference engine does), adopt it into the bucket view first.
        self._store.adopt_grad(p)
        self._on_ready([p])

    def _on_ready(self, params):
        if not self.require_backward_grad_sync or self._store is None:
            return
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        for p in params:
            b = self._bucket_of.get(id(p))
            if b is None or id(p) in self._ready_ids or not p.requires_grad:
                continue
            self._ready_ids.add(id(p))
            self._pending[b] -= 1
        while self._next_launch < len(self._buckets) and self._pending[self._next_launch] <= 0:
            self._launch(self._next_launch)
            self._next_launch += 1

    def _launch(self, b: int):
        lo, hi, _ = self._buckets[b]
        buf = self._store.grad_flat[lo:hi]
        t0 = self._timing_start() if self.timing else None
        tmp = None
        if self._comm_buf is not None:  # low-precision wire format, persistent mirror: no allocator traffic
            tmp = self._comm_buf[lo:hi]
            tmp.copy_(buf)
        wire = buf if tmp is None else tmp
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        w = dist.all_reduce(wire, op=op, group=self.process_group, async_op=True)
        self._works.append((w, buf, tmp))
        if t0 is not None:
            self._timing_end(w, t0, wire.numel() * wire.element_size())

    # ------------------------------------------------------------------ timing (opt-in)
    def _timing_start(self):
        if self._store.grad_flat.is_cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def _timing_end(self, w, t0, nbytes: int):
        if isinstance(t0, float):
            self._timings.append([nbytes, t0, w])  # resolved (host clock) when _finalize waits
            return
        if self._timing_stream is None:
            self._timing_stream = torch.cuda.Stream(device=self._store.grad_flat.device)
        ts = self._timing_stream
        e = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(ts):  # ts waits for the collective (no host sync), then stamps it
            w.wait()
            e.record(ts)
        self._timings.append((nbytes, t0, e))

    def pop_timing(self) -> List[tuple]:
        """This step's (bytes, start, end) per bucket, in launch order, and reset the list."""
        out = [tuple(t) for t in self._timings]
        self._timings = []
        return out

    def _finalize(self):
        while self._next_launch < len(self._buckets):
            self._launch(self._next_launch)
            self._next_launch += 1
        for w, buf, tmp in self._works:
            w.wait()
            for t in self._timings:  # gloo: completion stamped on the host clock when its wait returns
                if isinstance(t, list) and t[2] is w:
                    t[2] = time.perf_counter()
            if tmp is not None:
                buf.copy_(tmp)
            if not self._avg:
                buf.div_(self.world)
        self._works = []

    @property
    def transport(self) -> str:
        return f"torch-{dist.get_backend(self.process_group)}"

    # convenience passthroughs
    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)
