"""FusedAdamW: torch.optim.AdamW semantics (decoupled weight decay, bias correction;
`train/train_image_vit.py:270-276`) in ONE HIP launch over a model's flat parameter
buffer, with per-parameter lr / weight_decay from the param groups, optional gradient
clipping coefficient (clip_grad_norm_, `train_latent_vit_v2.py:133`) computed on device,
and the bf16 compute copy refreshed in the same pass.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import ops, runtime
from ._lib import AdamWSegment, check, lib


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 model=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.model = model
        self._flat = None
        self._m = self._v = None
        self._segs_dev = None
        self._seg_key = None
        self.grad_scale = 1.0        # e.g. 1/world after an all-reduce sum
        self.clip_coef: Optional[torch.Tensor] = None  # device scalar, consumed by the next step
        self._step_counter: Optional[torch.Tensor] = None  # graph mode (freeze_for_graph)
        self._frozen = None
        # eager mode: the segment table stays on the device between steps and the per-step bias-
        # correction step comes from a device counter (step = table step + *counter, advanced by one
        # stream-ordered launch per step) -- no per-step pinned allocation and H2D copy. Re-uploaded
        # when the segment set or any hyper-parameter changes.
        self.cache_table = True
        self._eager = None  # (device table, nseg, maxn, signature, counter, host steps of its last launch)
        # step_in_backward(): per-layer updates issued from the backward's gradient-ready hook
        self._inbw = False
        self._bw_done = set()     # ids of parameters already updated in the current backward
        self._bw_tables = {}      # parameter-set key -> (device table, nseg, maxn, signature, counter, tsegs, tiles)
        self._pgroup = None       # id(p) -> param group index

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics, plus: a clip coefficient left by clip_grad_norm_ for a step that was
        then skipped is dropped here, so it cannot scale the next step's unrelated gradients."""
        super().zero_grad(set_to_none=set_to_none)
        self.clip_coef = None
        if self.model is not None and getattr(self.model, "_fer_clip_coef", None) is not None:
            self.model._fer_clip_coef = None

    def _bind(self):
        flat = self.model.fer_flat() if self.model is not None else None
        if flat is None:
            raise RuntimeError("FusedAdamW needs model= (a fervit FerModule) to locate the flat buffers")
        if flat is not self._flat:
            self._flat = flat
            self._m = torch.zeros_like(flat.data)
            self._v = torch.zeros_like(flat.data)
        return flat

    # ---- torch.optim.AdamW-format state (checkpoints: utils/experiment_logger.py:121-145)
    def state_dict(self):
        """torch.optim.AdamW layout: per-parameter {'step', 'exp_avg', 'exp_avg_sq'} (moments
        copied out of the flat buffers) and the AdamW param-group keys, so a checkpoint written
        here resumes under torch.optim.AdamW and vice versa."""
        if self._flat is not None and self._m is not None:
            flat = self._flat
            for g in self.param_groups:
                for p in g["params"]:
                    st = self.state.get(p)
                    if st is None or id(p) not in flat.offsets:
                        continue
                    st["exp_avg"] = flat.view(p, self._m).detach().clone()
                    st["exp_avg_sq"] = flat.view(p, self._v).detach().clone()
        sd = super().state_dict()
        sd["state"] = {k: dict(v) for k, v in sd["state"].items()}  # detach from the live state
        sd["param_groups"] = [dict(g) for g in sd["param_groups"]]
        for st in sd["state"].values():
            if not torch.is_tensor(st.get("step", 0)):
                st["step"] = torch.tensor(float(st.get("step", 0)))
        for g in sd["param_groups"]:
            for k, v in (("amsgrad", False), ("maximize", False), ("foreach", None), ("capturable", False),
                         ("differentiable", False), ("fused", None)):
                g.setdefault(k, v)
        for g in self.param_groups:  # the live state keeps only the host step count
            for p in g["params"]:
                st = self.state.get(p)
                if st is not None:
                    st.pop("exp_avg", None)
                    st.pop("exp_avg_sq", None)
        return sd

    def load_state_dict(self, state_dict):
        self._eager = None
        self._bw_tables = {}
        super().load_state_dict(state_dict)
        flat = self._bind()
        with torch.no_grad():
            for g in self.param_groups:
                for p in g["params"]:
                    st = self.state.get(p)
                    if not st:
                        continue
                    if "exp_avg" in st:
                        flat.view(p, self._m).copy_(st.pop("exp_avg"))
                    if "exp_avg_sq" in st:
                        flat.view(p, self._v).copy_(st.pop("exp_avg_sq"))
                    if torch.is_tensor(st.get("step")):
                        st["step"] = int(st["step"].item())

    def freeze_for_graph(self, counter: torch.Tensor) -> None:
        """Graph mode (fervit.graph.StepGraph): the segment table is uploaded once and the
        AdamW step of every parameter becomes (its host step count now) + *counter, the device
        step counter the captured step advances. Call after the eager warm-up steps. A later
        change of a group's lr / weight_decay / betas / eps (an LR scheduler's step) is written
        into the same device table before the next replay (sync_graph_hparams)."""
        flat = self._bind()
        self._eager = None
        self._bw_tables = {}
        segs, maxn = self._segments(flat, bump=False)
        self._frozen = (self._upload(segs, flat), len(segs), maxn)
        # group of every segment (same walk as _segments), to rebuild the table with new hparams
        self._frozen_groups = [gi for gi, g in enumerate(self.param_groups) for p in g["params"] if p.grad is not None]
        self._frozen_segs = segs
        self._frozen_hp = self._hparams()
        self._step_counter = counter

    # ---- optimizer step inside the backward (opt-in)
    def step_in_backward(self, on: bool = True) -> "FusedAdamW":
        """Apply AdamW to each layer's parameters as soon as the layer's backward has written their
        gradients (runtime.grads_ready hook), on the weight-gradient stream behind that layer's weight
        gradients, instead of in one launch after the backward: the update (~0.5 ms of HBM-bound work on
        ViT-B/16) then runs beside the rest of the backward instead of after it, and step() only folds
        the host step counts. Bit-identical per parameter to step() (same kernel, same step, same
        arithmetic). Valid only when nothing between loss.backward() and step() changes the gradients
        -- the reference's train_epoch with grad_clip=None (`train/train_image_vit.py:121-131`): no
        clipping (step() raises if a clip coefficient is pending), no accumulation over several
        backward passes, no other gradient hook (DDP: the hook stands aside and step() updates
        everything as usual); under HIP-graph capture it stands aside as well."""
        if on and not self._inbw:
            runtime.register_grad_ready_hook(self._bw_hook)
        elif not on and self._inbw:
            runtime.remove_grad_ready_hook(self._bw_hook)
        self._inbw = on
        return self

    def _bw_hook(self, params) -> None:
        if not self._inbw or self._frozen is not None or len(runtime._HOOKS) > 1:
            return
        if torch.cuda.is_current_stream_capturing():
            return
        if self._pgroup is None:
            self._pgroup = {id(p): gi for gi, g in enumerate(self.param_groups) for p in g["params"]}
        flat = self._bind()
        if not flat.data.is_cuda:
            return
        if any(id(p) in self._bw_done for p in params if id(p) in self._pgroup and p.grad is not None):
            raise RuntimeError("FusedAdamW.step_in_backward: a second backward reached parameters already updated "
                               "since the last step() (gradient accumulation is not supported in this mode)")
        ps = [p for p in params if id(p) in self._pgroup and p.grad is not None]
        if not ps:
            return
        segs, maxn = [], 0
        for p in ps:
            if p.grad.data_ptr() != flat.grad_views[id(p)].data_ptr():
                return  # a foreign .grad tensor: leave this layer to step()
        for p in ps:
            g = self.param_groups[self._pgroup[id(p)]]
            st = self.state[p]
            st["step"] = st.get("step", 0) + 1
            b1, b2 = g["betas"]
            segs.append((flat.offsets[id(p)], p.numel(), g["lr"], g["weight_decay"], b1, b2, g["eps"], st["step"]))
            maxn = max(maxn, p.numel())
        key = tuple(id(p) for p in ps)
        sig = tuple(x[:7] for x in segs)
        steps = tuple(x[7] for x in segs)
        e = self._bw_tables.get(key)
        # reuse the resident table only if every parameter's host step moved by exactly one since the
        # table's last launch (its device step = table step + counter advances by one per reuse);
        # anything else -- another update path, a different subset, graph replays -- rebuilds it
        advance = e is not None and e[3] == sig and all(s == t + 1 for s, t in zip(steps, e[7]))
        if not advance:
            dev = self._upload(segs, flat)
            counter = torch.zeros(1, dtype=torch.int64, device=flat.data.device)
            tsegs, tiles = flat.half_t_segments(ps)
            e = (dev, len(segs), maxn, sig, counter, tsegs, tiles, steps)
        dev, nseg, maxn, _, counter, tsegs, tiles, _ = e
        if tsegs is None and flat.half_t is not None:  # the transposed copies appeared after the table was built
            tsegs, tiles = flat.half_t_segments(ps)
        self._bw_tables[key] = (dev, nseg, maxn, sig, counter, tsegs, tiles, steps)
        self._eager = None  # these parameters' steps moved outside step()'s resident table
        half = flat.bf16()

        def launch():
            if advance:
                check(lib().fer_step_advance(counter.data_ptr(), ops.stream()), "adamw step")
            check(lib().fer_adamw(flat.data.data_ptr(), flat.grad.data_ptr(), self._m.data_ptr(), self._v.data_ptr(),
                                  half.data_ptr(), dev.data_ptr(), nseg, maxn, float(self.grad_scale), None,
                                  counter.data_ptr(), ops.stream()), "adamw")
            if tsegs is not None and flat.half_t is not None:
                check(lib().fer_transpose_bf16_segments(half.data_ptr(), flat.half_t.data_ptr(), tsegs.data_ptr(),
                                                        tsegs.shape[0], tiles, ops.stream()), "transpose")

        runtime.WGRAD.run(launch, flat.grad)
        self._bw_done.update(key)

    def _hparams(self):
        return [(g["lr"], g["weight_decay"], tuple(g["betas"]), g["eps"]) for g in self.param_groups]

    def sync_graph_hparams(self) -> bool:
        """Graph mode: if any group's hyper-parameters changed since the table was uploaded (e.g.
        CosineAnnealingLR.step() at an epoch end, `train/train_latent_vit_v2.py:368-370`), rewrite
        the captured segment table in place (a stream-ordered copy ahead of the replay: the
        replayed AdamW node reads it from device memory). Returns True when it rewrote it."""
        if self._frozen is None:
            return False
        hp = self._hparams()
        if hp == self._frozen_hp:
            return False
        if len(hp) != len(self._frozen_hp):
            raise RuntimeError("FusedAdamW: param groups changed under a captured StepGraph; release() it first")
        segs = []
        for gi, (off, n, _lr, _wd, _b1, _b2, _eps, step) in zip(self._frozen_groups, self._frozen_segs):
            g = self.param_groups[gi]
            b1, b2 = g["betas"]
            segs.append((off, n, g["lr"], g["weight_decay"], b1, b2, g["eps"], step))
        self._frozen[0].copy_(self._upload(segs, self._flat), non_blocking=True)
        self._frozen_segs = segs
        self._frozen_hp = hp
        return True

    def unfreeze(self) -> None:
        """Leave graph mode (StepGraph.release): the replays' device step count is folded into
        every parameter's host 'step', so state_dict() and later eager steps continue the bias
        correction where the replays left it."""
        if self._step_counter is not None:
            n = int(self._step_counter.item())
            if n:
                for g in self.param_groups:
                    for p in g["params"]:
                        st = self.state.get(p)
                        if st is not None and "step" in st:
                            st["step"] = st["step"] + n
        self._frozen = None
        self._step_counter = None
        self._eager = None
        self._bw_tables = {}

    def _segments(self, flat, bump: bool):
        segs = []
        maxn = 0
        for g in self.param_groups:
            b1, b2 = g["betas"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if bump:
                    st["step"] = st.get("step", 0) + 1
                n = p.numel()
                maxn = max(maxn, n)
                segs.append((flat.offsets[id(p)], n, g["lr"], g["weight_decay"], b1, b2, g["eps"],
                             st.get("step", 0)))
                if p.grad.data_ptr() != flat.grad_views[id(p)].data_ptr():
                    flat.grad_views[id(p)].copy_(p.grad)
        return segs, maxn

    @staticmethod
    def _upload(segs, flat):
        """Segment table -> device through pinned memory, stream-ordered: a pageable blocking
        copy would make the host wait for the whole step's kernels every optimizer step, and
        the GPU then idle while the next step's first launches are issued."""
        arr = (AdamWSegment * len(segs))(*[AdamWSegment(*s) for s in segs])
        host = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))),
                                dtype=torch.uint8)
        if flat.data.is_cuda:
            host = host.pin_memory()  # the caching host allocator keeps it until the copy is done
            return host.to(flat.data.device, non_blocking=True)
        return host.to(flat.data.device)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        flat = self._bind()
        runtime.WGRAD.sync()  # weight gradients of the last backward (normally joined already)
        _close_reduce_window()
        if self._bw_done:  # step_in_backward: most (usually all) parameters were updated in the backward
            done, self._bw_done = self._bw_done, set()
            if self._take_clip() is not None:
                raise RuntimeError("FusedAdamW.step_in_backward: gradient clipping between backward and step() "
                                   "cannot apply to updates already made; disable step_in_backward")
            rest = [p for g in self.param_groups for p in g["params"] if p.grad is not None and id(p) not in done]
            if rest:
                self._step_subset(flat, rest)
            flat.mark_half_fresh(refresh=False)  # (each layer's transposed copies were refreshed with it)
            return loss
        if self._frozen is not None:  # graph mode: static segments, device step counter
            dev, nseg, maxn = self._frozen
            half = flat.bf16()
            check(lib().fer_adamw(flat.data.data_ptr(), flat.grad.data_ptr(), self._m.data_ptr(),
                                  self._v.data_ptr(), half.data_ptr(), dev.data_ptr(), nseg, maxn,
                                  float(self.grad_scale), ops.ptr(self._take_clip()),
                                  self._step_counter.data_ptr(), ops.stream()), "adamw")
            flat.mark_half_fresh()
            return loss
        segs, maxn = self._segments(flat, bump=True)
        if not segs:
            return loss
        counter = None
        sig = tuple(s[:7] for s in segs)
        steps = tuple(s[7] for s in segs)
        e = self._eager
        if (self.cache_table and e is not None and e[3] == sig and flat.data.is_cuda
                and all(s == t + 1 for s, t in zip(steps, e[5]))):
            # same segments and hyper-parameters as the resident table, every step bumped by one since
            dev, counter = e[0], e[4]
            check(lib().fer_step_advance(counter.data_ptr(), ops.stream()), "adamw step")
            self._eager = e[:5] + (steps,)
        else:
            dev = self._upload(segs, flat)
            self._eager = None
            if self.cache_table and flat.data.is_cuda:
                counter = torch.zeros(1, dtype=torch.int64, device=flat.data.device)
                self._eager = (dev, len(segs), maxn, sig, counter, steps)
        self._segs_dev = dev
        half = flat.bf16()
        check(lib().fer_adamw(flat.data.data_ptr(), flat.grad.data_ptr(), self._m.data_ptr(), self._v.data_ptr(),
                              half.data_ptr(), dev.data_ptr(), len(segs), maxn, float(self.grad_scale),
                              ops.ptr(self._take_clip()), ops.ptr(counter), ops.stream()), "adamw")
        flat.mark_half_fresh()
        return loss

    def _step_subset(self, flat, params) -> None:
        """One eager update of `params` only (the ones step_in_backward's hook did not reach)."""
        self._eager = None  # steps move outside the resident table (the per-layer tables check theirs)
        ids = {id(p) for p in params}
        segs, maxn = [], 0
        for g in self.param_groups:
            b1, b2 = g["betas"]
            for p in g["params"]:
                if id(p) not in ids:
                    continue
                st = self.state[p]
                st["step"] = st.get("step", 0) + 1
                segs.append((flat.offsets[id(p)], p.numel(), g["lr"], g["weight_decay"], b1, b2, g["eps"], st["step"]))
                maxn = max(maxn, p.numel())
                if p.grad.data_ptr() != flat.grad_views[id(p)].data_ptr():
                    flat.grad_views[id(p)].copy_(p.grad)
        dev = self._upload(segs, flat)
        self._segs_dev = dev
        half = flat.bf16()
        check(lib().fer_adamw(flat.data.data_ptr(), flat.grad.data_ptr(), self._m.data_ptr(), self._v.data_ptr(),
                              half.data_ptr(), dev.data_ptr(), len(segs), maxn, float(self.grad_scale), None, None,
                              ops.stream()), "adamw")
        tsegs, tiles = flat.half_t_segments(params)
        if tsegs is not None and flat.half_t is not None:
            check(lib().fer_transpose_bf16_segments(half.data_ptr(), flat.half_t.data_ptr(), tsegs.data_ptr(),
                                                    tsegs.shape[0], tiles, ops.stream()), "transpose")

    def _take_clip(self) -> Optional[torch.Tensor]:
        """The pending clip coefficient (set by clip_grad_norm_ through `optimizer=` or left on
        the model), consumed by this step."""
        coef = self.clip_coef
        if coef is None and self.model is not None:
            coef = getattr(self.model, "_fer_clip_coef", None)
        self.clip_coef = None
        if self.model is not None and hasattr(self.model, "_fer_clip_coef"):
            self.model._fer_clip_coef = None
        return coef


def _close_reduce_window() -> None:
    """Queued bias / LayerNorm gradient sums of a backward that raised (layers._ReduceDefer)."""
    from .layers import REDUCE

    REDUCE.close_if_open()


def clip_grad_norm_(model, max_norm: float, sq_scale: float = 1.0, optimizer: Optional[FusedAdamW] = None
                    ) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ (`train/train_latent_vit_v2.py:133`) on the model's flat
    grad buffer without a host synchronisation: total = ||g||_2 over every gradient, coef =
    min(1, max_norm / (total + 1e-6)). The gradients are not rescaled here: the coefficient is
    handed to the fused optimizer (`optimizer.clip_coef`, and `model._fer_clip_coef` for a
    FusedAdamW bound to this model), whose next step multiplies every gradient by it -- the
    same arithmetic as torch's in-place `g *= coef` followed by AdamW. Returns the total norm
    (device scalar), as torch does. Like torch, only parameters with a gradient count: a
    parameter whose `.grad` is None (never written, or dropped by zero_grad(set_to_none=True)
    after an earlier backward wrote its slot) contributes nothing -- FlatParams.settle_grads
    zeroes such stale slots and copies foreign `.grad` tensors into the flat buffer first."""
    flat = model.fer_flat()
    runtime.WGRAD.sync()
    _close_reduce_window()
    flat.settle_grads()
    out = torch.empty(2, dtype=torch.float32, device=flat.grad.device)
    ws = ops.WS.get(4 * 4096, flat.grad.device, slot=3)
    check(lib().fer_sumsq(flat.grad.data_ptr(), flat.numel, out.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                          ops.stream()), "sumsq")
    check(lib().fer_clip_coef(out.data_ptr(), sq_scale, float(max_norm), out[1:].data_ptr(), ops.stream()), "clip")
    coef = out[1:]
    model._fer_clip_coef = coef
    if optimizer is not None:
        optimizer.clip_coef = coef
    if sq_scale == 1.0:
        return out[0].sqrt()
    return (out[0] * sq_scale).sqrt()
