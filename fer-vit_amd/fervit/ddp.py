"""Data-parallel training over RCCL (xGMI) — the reference trains single-device
(`train/train_image_vit.py:183`); this is the greenfield DDP layer of SURVEY §8(e).

One process per GPU. Gradients live in the model's flat fp32 grad buffer, so a bucket
is just a contiguous slice of it (no pack/unpack copies). Buckets are cut in reverse
flat order (the order backward finishes layers), only over trainable parameters, at
~bucket_cap_mb. When a layer's backward has written its gradients, the layer calls
`runtime.grads_ready`; the reducer records an event on the compute stream and, once a
bucket is complete, issues its all-reduce (AVG on RCCL, SUM + scale on gloo) on a side
stream, overlapping communication with the remaining backward. A callback queued on the
autograd engine makes the compute stream wait for every bucket before backward returns,
so the optimizer always sees averaged gradients.

Under fervit.graph.StepGraph capture the same calls are recorded: the hooks and the end-of-backward
callback run once, at capture time, and the captured graph holds the bucket casts, the RCCL
all-reduce kernels on the side stream and the joins -- a replayed DDP step issues no host work per
bucket (the launch-bound configurations: hybrid / expression-aware w+ models, 48 px images).

`grad_dtype=torch.bfloat16` halves the bytes on the wire (ViT-B: 172 MB instead of 343 MB
per step): each bucket is cast into a persistent bf16 communication buffer on the side stream
(libfervit cast kernel), all-reduced in bf16, and cast back into the fp32 flat gradient before
the optimizer. The sum is then rounded to bf16 at every reduction hop (like torch DDP's
bf16 compression hook); the default stays fp32.

Modules that are not fervit FerModules (e.g. CPU toy models in the gloo tests) get the
same reducer fed by post-accumulate-grad hooks that copy p.grad into the flat buffer.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from . import runtime
from .runtime import FlatParams


class _Bucket:
    __slots__ = ("params", "lo", "hi", "pending", "work", "launched")

    def __init__(self, params, lo, hi):
        self.params = params
        self.lo, self.hi = lo, hi
        self.pending = set()
        self.work = None
        self.launched = False


class Reducer:
    def __init__(self, flat: FlatParams, params: List[nn.Parameter], group=None, bucket_cap_mb: float = 32.0,
                 grad_dtype: torch.dtype = torch.float32):
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("grad_dtype must be torch.float32 or torch.bfloat16")
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        cap = int(bucket_cap_mb * 1024 * 1024 / 4)
        trainable = {id(p) for p in params if p.requires_grad}
        order = sorted(flat.params, key=lambda p: flat.offsets[id(p)], reverse=True)
        self.buckets: List[_Bucket] = []
        cur: List[nn.Parameter] = []
        size = 0
        for p in order:
            if id(p) not in trainable:
                if cur:
                    self._close(cur)
                cur, size = [], 0
                continue
            cur.append(p)
            size += p.numel()
            if size >= cap:
                self._close(cur)
                cur, size = [], 0
        if cur:
            self._close(cur)
        self.where: Dict[int, _Bucket] = {id(p): b for b in self.buckets for p in b.params}
        self.cuda = flat.grad.is_cuda
        self.side = torch.cuda.Stream(device=flat.grad.device) if self.cuda else None
        self.comm = (torch.empty(flat.grad.numel(), dtype=torch.bfloat16, device=flat.grad.device)
                     if grad_dtype == torch.bfloat16 else None)
        self.armed = False
        self.queued = False

    def _close(self, ps):
        lo = min(self.flat.offsets[id(p)] for p in ps)
        hi = max(self.flat.offsets[id(p)] + p.numel() for p in ps)
        self.buckets.append(_Bucket(list(ps), lo, hi))

    # ---- per iteration
    def prepare(self):
        for b in self.buckets:
            b.pending = {id(p) for p in b.params}
            b.work = None
            b.launched = False
        self.armed = True
        self.queued = False

    def on_ready(self, params):
        if not self.armed:
            return
        if not self.queued:
            self.queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self.finalize)
        for p in params:
            b = self.where.get(id(p))
            if b is None:
                continue
            b.pending.discard(id(p))
            if not b.pending and not b.launched:
                self._launch(b)

    def _launch(self, b: _Bucket):
        b.launched = True
        view = self.flat.grad[b.lo:b.hi]
        if self.cuda:
            self.side.wait_stream(torch.cuda.current_stream(view.device))
            wg = runtime.WGRAD.stream(view.device)  # weight gradients finish on their own stream
            # Wait on it whenever the weight gradients actually run there: eagerly, and under
            # HIP-graph capture with WGRAD.in_capture (the side stream is then a forked branch of
            # the captured graph). With the stream off (capture without in_capture, or disabled)
            # they ran on the compute stream, which self.side already waited for above.
            if wg is not None and not runtime.WGRAD._off():
                self.side.wait_stream(wg)
            with torch.cuda.stream(self.side):
                b.work = self._allreduce(self._to_wire(b, view))
        else:
            b.work = self._allreduce(self._to_wire(b, view))

    def _to_wire(self, b: _Bucket, view):
        if self.comm is None:
            return view
        wire = self.comm[b.lo:b.hi]
        if view.is_cuda:
            from . import ops
            ops.cast_bf16(view, out=wire)
        else:  # CPU toy models of the gloo tests
            wire.copy_(view)
        return wire

    def _from_wire(self, b: _Bucket):
        if self.comm is None:
            return
        view, wire = self.flat.grad[b.lo:b.hi], self.comm[b.lo:b.hi]
        if view.is_cuda:
            from . import ops
            ops.cast_f32(wire, out=view)
        else:
            view.copy_(wire)

    def _allreduce(self, view):
        if self.backend == "nccl":
            return dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        return dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finalize(self):
        # parameters that produced no gradient this step: reduce zeros so ranks agree
        for b in self.buckets:
            if not b.launched:
                for p in b.params:
                    if id(p) in b.pending:
                        self.flat.grad_views[id(p)].zero_()
                        self.flat.attach(p)
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
        if self.cuda:
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(self.side)
        for b in self.buckets:
            self._from_wire(b)
        if self.backend != "nccl":
            for b in self.buckets:
                self.flat.grad[b.lo:b.hi].div_(self.world)
        self.armed = False


class DistributedDataParallel(nn.Module):
    """Wrap a model; `forward` arms the reducer, backward all-reduces gradient buckets."""

    def __init__(self, module: nn.Module, bucket_cap_mb: float = 32.0, process_group=None,
                 broadcast_params: bool = True, grad_dtype: torch.dtype = torch.float32):
        super().__init__()
        self.module = module
        self.group = process_group
        from .module import FerModule

        self.is_fer = isinstance(module, FerModule)
        if self.is_fer:
            flat = module.fer_flat()
        else:
            flat = FlatParams(list(module.parameters()))
            for p in flat.params:
                if p.requires_grad:
                    p.register_post_accumulate_grad_hook(self._hook)
        self.flat = flat
        if broadcast_params:
            with torch.no_grad():
                dist.broadcast(flat.data, src=0, group=process_group)
        self.reducer = Reducer(flat, list(module.parameters()), process_group, bucket_cap_mb, grad_dtype)
        runtime.register_grad_ready_hook(self.reducer.on_ready)

    def _hook(self, p):
        gv = self.flat.grad_views[id(p)]
        if p.grad.data_ptr() != gv.data_ptr():
            gv.copy_(p.grad)
            p.grad = gv
        self.reducer.on_ready([p])

    def forward(self, *args, **kwargs):
        if torch.is_grad_enabled():
            self.reducer.prepare()
        return self.module(*args, **kwargs)

    def __del__(self):
        try:
            runtime.remove_grad_ready_hook(self.reducer.on_ready)
        except Exception:
            pass
