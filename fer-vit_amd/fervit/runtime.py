"""Runtime state: precision mode, dropout seed stream, flat parameter storage.

Flat parameter storage (one per model): every parameter of a model lives in ONE
contiguous fp32 buffer (64-element aligned offsets), its gradient in ONE fp32
grad buffer with the same offsets, and the bf16 compute copy in ONE bf16 buffer.
So the optimizer is one fused launch, the bf16 refresh is one cast, and DDP
all-reduces contiguous buckets of the grad buffer with no packing copies.
`p.data` / `p.grad` of each nn.Parameter are views into these buffers, so every
torch API (state_dict, optimizers, clip_grad_norm_) keeps working unchanged.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional

import torch

ALIGN = 64

_state = threading.local()


def default_precision() -> str:
    return os.environ.get("FERVIT_PRECISION", "bf16")


class _Seeds:
    def __init__(self):
        self.base = None
        self.counter = 0

    def next(self) -> int:
        if self.base is None:
            self.base = (torch.initial_seed() * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        # splitmix64: every dropout site gets a fully mixed 64-bit key (the device hash only
        # xors/adds the key into the element counter before its finaliser, csrc/common.h)
        self.counter += 1
        m = 0xFFFFFFFFFFFFFFFF
        z = (self.base + self.counter * 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        return z ^ (z >> 31)


SEEDS = _Seeds()


def manual_seed(seed: int) -> None:
    SEEDS.base = (int(seed) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    SEEDS.counter = 0


def next_seed() -> int:
    return SEEDS.next()


class FlatParams:
    """Flat fp32 / grad / bf16 storage for a list of parameters (see module doc)."""

    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = list(params)
        self.offsets: Dict[int, int] = {}
        off = 0
        for p in self.params:
            self.offsets[id(p)] = off
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = max(off, ALIGN)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.device = dev
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.half: Optional[torch.Tensor] = None
        self.half_version = -1
        self._checked = False  # version signature already compared during this forward pass
        self._passes = False  # set by the owning module's forward (begin_pass): enables the cache
        self.half_t: Optional[torch.Tensor] = None  # transposed bf16 copies of the 2-D params
        self._tsegs: Optional[torch.Tensor] = None
        self._ttiles = 0
        self._written = set()  # ids of parameters whose grad slot a backward has written
        self.owner_active = False  # inside the owning module's forward (FerModule hooks)
        with torch.no_grad():
            for p in self.params:
                v = self.view(p)
                v.copy_(p.data)
                p.data = v
        self.grad_views = {id(p): self.grad_view(p) for p in self.params}

    def view(self, p, buf=None):
        buf = self.data if buf is None else buf
        o = self.offsets[id(p)]
        return buf[o:o + p.numel()].view(p.shape)

    def grad_view(self, p):
        return self.view(p, self.grad)

    # ---- bf16 compute copy
    def bf16(self) -> torch.Tensor:
        """bf16 shadow of the fp32 buffer, refreshed when any parameter changed in place
        (version counter of the shared storage) or when marked stale."""
        from . import ops

        if self.half is None:
            self.half = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
        if self._passes and self._checked and self.half_version >= 0:
            return self.half
        v = self.version()
        self._checked = True
        if v != self.half_version:
            ops.cast_bf16(self.data, self.half)
            self.half_version = v
            self.refresh_half_t()
        return self.half

    def begin_pass(self) -> None:
        """Start of the owning model's forward: the next bf16() compares the version signature
        (O(#params) host work) once; every other weight fetch of the pass -- and of its
        backward -- reuses that result instead of re-summing per GEMM launch."""
        self._passes = True
        self._checked = False

    def version(self) -> int:
        # in-place updates through a Parameter bump that Parameter's own counter
        # (not the flat base's), so the signature is the sum over parameters.
        return self.data._version + sum(p._version for p in self.params)

    def mark_half_fresh(self, refresh: bool = True):
        """Called by the fused optimizer right after it rewrote the bf16 copy (same stream):
        the transposed copies follow in the same stream order (and the same captured graph);
        refresh=False when the optimizer refreshed them per parameter set already."""
        self.half_version = self.version()
        self._checked = True
        if refresh:
            self.refresh_half_t()

    def half_t_segments(self, params):
        """(device segment table, tile count) of the transposed-copy refresh for the 2-D parameters in
        `params` (None when there are none or no transposed copy exists yet)."""
        if self.half_t is None:
            return None, 0
        segs, tiles = [], 0
        for q in params:
            if q.dim() == 2:
                r, c = q.shape
                segs.append((self.offsets[id(q)], r, c, tiles))
                tiles += -(-r // 64) * -(-c // 64)
        if not segs:
            return None, 0
        return torch.tensor(segs, dtype=torch.int64).to(self.device), tiles

    def half_view(self, p):
        return self.view(p, self.bf16())

    # ---- transposed bf16 copies (dgrad operands, K-contiguous)
    def refresh_half_t(self):
        if self.half_t is None or self.half is None:
            return
        from ._lib import check, lib
        from . import ops

        check(lib().fer_transpose_bf16_segments(self.half.data_ptr(), self.half_t.data_ptr(), self._tsegs.data_ptr(),
                                                self._tsegs.shape[0], self._ttiles, ops.stream()), "transpose")

    def half_t_view(self, p):
        """bf16 W^T ([cols][rows]) of a 2-D parameter, kept in step with the bf16 shadow: one
        batched transpose launch per refresh of the shadow (optimizer step or cast)."""
        if self.half_t is None:
            segs, tiles = [], 0
            for q in self.params:
                if q.dim() == 2:
                    r, c = q.shape
                    segs.append((self.offsets[id(q)], r, c, tiles))
                    tiles += -(-r // 64) * -(-c // 64)
            self._tsegs = torch.tensor(segs, dtype=torch.int64).to(self.device)
            self._ttiles = tiles
            self.bf16()
            self.half_t = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            self.refresh_half_t()
        else:
            self.bf16()
        if p.dim() != 2:
            raise ValueError("half_t_view: 2-D parameters only")
        o = self.offsets[id(p)]
        r, c = p.shape
        return self.half_t[o:o + p.numel()].view(c, r)

    # ---- gradient side channel
    def settle_grads(self) -> None:
        """Make the flat grad buffer equal torch's view of the gradients before a whole-buffer
        reduction (clip_grad_norm_): a slot written in an earlier backward whose parameter's
        `.grad` is now None is zeroed (torch skips such parameters), and a foreign `.grad`
        tensor (assigned by user code) is copied into its slot."""
        for p in self.params:
            g = p.grad
            if g is None:
                if id(p) in self._written:
                    self.grad_views[id(p)].zero_()
                    self._written.discard(id(p))
            elif g.data_ptr() != self.grad_views[id(p)].data_ptr():
                with torch.no_grad():
                    self.grad_views[id(p)].copy_(g)
                self._written.add(id(p))

    def grad_target(self, p) -> (torch.Tensor, bool):
        """(view to write p's gradient into, accumulate?) following torch semantics:
        p.grad None -> overwrite; p.grad is our view -> accumulate; foreign tensor ->
        copy it into the view, then accumulate."""
        self._written.add(id(p))
        gv = self.grad_views[id(p)]
        g = p.grad
        if g is None:
            return gv, False
        if g.data_ptr() == gv.data_ptr():
            return gv, True
        with torch.no_grad():
            gv.copy_(g)
        return gv, True

    def attach(self, p):
        gv = self.grad_views[id(p)]
        if p.grad is None or p.grad.data_ptr() != gv.data_ptr():
            p.grad = gv


_HOOKS: List = []


def register_grad_ready_hook(fn) -> None:
    _HOOKS.append(fn)


def remove_grad_ready_hook(fn) -> None:
    if fn in _HOOKS:
        _HOOKS.remove(fn)


def grads_ready(params) -> None:
    """Layer backward finished writing these parameters' gradients."""
    for h in list(_HOOKS):
        h(params)


# ------------------------------------------------------------ weight-gradient stream
class _WgradStream:
    """Weight gradients (dW = dY^T X) on a second HIP stream.

    A layer's backward is a chain dY -> dX through dgrad GEMMs; the weight gradients hang off
    that chain and nothing in the backward reads them. Issued on a side stream (after an event
    on the compute stream), their split-K GEMMs take the CUs the dgrad GEMMs leave idle in their
    last tile round (ViT-B: the N=768 GEMMs are 591 256x256 tiles = 2.31 rounds of 256 CUs).
    Inputs are marked with record_stream so the caching allocator does not hand their memory
    to the compute stream while the side stream reads it, and the first use in a backward
    queues an autograd-engine callback that makes the compute stream wait for the side stream
    before backward returns (optimizer, clipping and user code then see finished gradients).
    Under HIP-graph capture (StepGraph) the side stream forks from the capturing stream through
    the same event wait and is joined back by the same callback, so the captured graph keeps the
    two branches -- with `in_capture` only: measured on the graph-replayed configs (r03m, one box)
    it did not pay (w+ latent ViT 3.07 -> 3.04 ms, hybrid 7.09 -> 7.22 ms, 48 px ImageViT 1.65 ->
    1.75 ms), so captured steps keep one branch. `enabled = False` puts the weight gradients on the
    compute stream (the bench's isolated GEMM probe)."""

    def __init__(self):
        self.streams = {}
        self.join_queued = False
        self.enabled = True
        self.in_capture = False
        # CU mask of the side stream (list of 32-bit words, bit i = CU i; None: every CU). Set before
        # the first backward; the stream is created on first use (fer_stream_create_cu_mask). A masked
        # stream is a BLOCKING stream (hipExtStreamCreateWithCUMask takes no flags): beside work on the
        # legacy null stream it serialises with it, so run the step on a non-blocking stream when a mask
        # is set (tools/step_ab.py does).
        self.cu_mask: Optional[List[int]] = None
        self._handles = {}
        self._retired = []  # masked handles of earlier reset()s, never destroyed (see reset)

    def _make(self, dev):
        if not self.cu_mask:
            return torch.cuda.Stream(device=dev)
        import ctypes

        from ._lib import check, lib

        words = (ctypes.c_uint32 * len(self.cu_mask))(*[int(w) & 0xFFFFFFFF for w in self.cu_mask])
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(lib().fer_stream_create_cu_mask(words, len(self.cu_mask), 0, ctypes.byref(h)), "wgrad stream")
        self._handles[dev] = h.value
        return torch.cuda.ExternalStream(h.value, device=dev)

    def reset(self):
        """Drop the side streams (e.g. after changing cu_mask); call with no backward in flight.

        A CU-masked stream's handle is NOT destroyed: tensors such as flat.grad carry it from
        record_stream(), and the caching allocator records an event on it whenever such a tensor is
        freed, however much later -- on a destroyed handle that is an invalid-handle error or a
        silently reused one. The handles stay alive for the life of the process (_retired)."""
        if self.streams:
            torch.cuda.synchronize()
        self.streams = {}
        self._retired.extend(self._handles.values())
        self._handles = {}

    def _off(self) -> bool:
        return not self.enabled or (not self.in_capture and torch.cuda.is_current_stream_capturing())

    def stream(self, device):
        return self.streams.get(device)

    def run(self, fn, *inputs):
        dev = inputs[0].device
        if self._off():
            return fn()
        main = torch.cuda.current_stream(dev)
        side = self.streams.get(dev)
        if side is None:
            side = self.streams[dev] = self._make(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            out = fn()
        for t in inputs:
            t.record_stream(side)
        if not self.join_queued:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._join)
                self.join_queued = True
            except RuntimeError:  # not inside a backward pass: join right away
                self._join()
        return out

    def _join(self):
        self.join_queued = False
        self.sync()

    def sync(self):
        """The current (compute) stream waits for every weight gradient issued so far."""
        if not self.streams or (not self.in_capture and torch.cuda.is_current_stream_capturing()):
            return
        for dev, side in self.streams.items():
            torch.cuda.current_stream(dev).wait_stream(side)


WGRAD = _WgradStream()
