"""Autograd functions of the hot path. Each forward/backward is a fixed sequence of
libfervit kernel launches (ops.py); parameter gradients are written by the kernels
straight into the model's flat fp32 gradient buffer (runtime.FlatParams) and then
attached as `p.grad`, so autograd never allocates or accumulates them.

Layer math (reference):
  PostNormLayerFn  nn.TransformerEncoderLayer(norm_first=False) (`image_vit.py:101-113`,
                   `latent_vit.py:24-31`): x1 = LN1(x + Drop(SA(x))); out = LN2(x1 + Drop(FFN(x1)))
  PreNormBlockFn   timm Block (`hybrid_latent_vit.py:227-233`): x + Attn(LN1 x); x + MLP(LN2 x)
  AdapterFn        AdapterModule (`hybrid_latent_vit.py:249-265`)
  PatchTokensFn    PatchEmbedding + CLS/pos + Dropout (`image_vit.py:34-44,148-156`)
  LatentTokensFn   input_proj + CLS/pos (`latent_vit.py:38-44`, `hybrid_latent_vit.py:212-222`)
  HeadFn           LN on CLS + [Dropout] + Linear (`image_vit.py:161-164`, `latent_vit.py:46-47`,
                   `hybrid_latent_vit.py:236-237`)
  WplusFn          SPE -> LWN -> LEAM (`latent_vit_v2.py:82-84`)
"""
from __future__ import annotations

import functools
from dataclasses import dataclass
from typing import List, Optional, Sequence

import os

import torch

from . import ops
from . import runtime
from ._lib import check, lib
from .runtime import WGRAD, FlatParams, grads_ready, next_seed


@dataclass
class LayerCfg:
    B: int
    N: int
    H: int
    act: str = "gelu"
    dropout: float = 0.0
    eps: float = 1e-5
    save: bool = True


def _weight(flat: FlatParams, p: torch.nn.Parameter, dt: torch.dtype) -> torch.Tensor:
    """Matrix operand in the compute dtype (bf16 shadow or the fp32 master)."""
    return flat.half_view(p) if dt == torch.bfloat16 else p.data


def _dgrad(flat: FlatParams, dy: torch.Tensor, p: torch.nn.Parameter, dt: torch.dtype, **kw) -> torch.Tensor:
    """dx = dy W (nn.Linear input gradient). bf16 reads the transposed shadow W^T as a
    K-contiguous operand (a forward-layout GEMM, 10-20 % faster than the MN-operand read);
    fp32 (parity path) reads the master weight as an MN operand."""
    if dt == torch.bfloat16:
        return ops.linear_fwd(dy, flat.half_t_view(p), **kw)
    return ops.linear_dgrad(dy, p.data, **kw)


def _targets(flat: FlatParams, params: Sequence[torch.nn.Parameter], needs: Sequence[bool]):
    """Gradient destinations + one accumulate flag shared by the group."""
    outs, accs = [], []
    for p, n in zip(params, needs):
        if n:
            gv, acc = flat.grad_target(p)
            outs.append(gv)
            accs.append(acc)
        else:
            outs.append(None)
    if accs and any(accs) and not all(accs):
        for gv, p, n in zip(outs, params, needs):
            if n and p.grad is None:
                gv.zero_()
        return outs, True
    return outs, bool(accs and accs[0])


class _ReduceDefer:
    """Deferred bias / LayerNorm gradient reductions over one backward pass (csrc/misc.hip
    fer_reduce_defer). Inside a layer's backward the LayerNorm / attention / fused-GEMM column
    partials go to a persistent arena and their fixed-order sums (`part_reduce`, ~4-5 per layer,
    each a short dependent launch on the compute stream) are queued; the end of the backward (an
    autograd-engine callback), a gradient-ready hook (DDP buckets) or a full queue runs them as ONE
    launch. Bit-identical to the immediate reductions. Only the layer functions below open the
    window (they write gradients into the flat buffer, which nothing reads before the backward
    ends); every other caller of the same ops keeps the immediate path. `enabled` turns it off (tests);
    the arena is 64 MB (a full arena flushes) and csrc takes partial sets up to 2 MB (small-token
    configs)."""

    def __init__(self):
        self.enabled = True
        self.mb = 64
        self.arena: Optional[torch.Tensor] = None
        self.open = False
        self.owner = -1  # autograd graph task whose end-of-backward callback closes the window
        self.windows = 0  # backward passes that deferred (tests)

    def begin(self, device) -> bool:
        if not self.enabled or device is None or device.type != "cuda":
            return False
        task = torch._C._current_graph_task_id()
        if self.open and task != self.owner:
            # the window's backward ended without running its callback (torch drops queued
            # callbacks when a backward raises): run what it queued, then open a fresh window
            self._end()
        if not self.open:
            if self.arena is None or self.arena.device != device:
                if torch.cuda.is_current_stream_capturing():
                    return False  # allocate in an eager step first (StepGraph warm-up)
                self.arena = torch.empty(self.mb << 18, dtype=torch.float32, device=device)
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._end)
            except RuntimeError:  # not inside a backward pass
                return False
            self.open = True
            self.owner = task
            self.windows += 1
        check(lib().fer_reduce_defer(1, self.arena.data_ptr(), self.arena.numel() * 4, ops.stream()), "reduce_defer")
        return True

    def pause(self) -> None:
        check(lib().fer_reduce_defer(2, None, 0, None), "reduce_defer")

    def flush(self) -> None:
        if self.open:
            check(lib().fer_reduce_flush(), "reduce_flush")

    def _end(self) -> None:
        self.open = False
        self.owner = -1
        check(lib().fer_reduce_defer(0, None, 0, None), "reduce_defer")

    def close_if_open(self) -> None:
        """Readers of the gradients (optimizer step, clipping) outside a backward: a window still
        open here lost its callback to an exception in its backward -- run its queued sums now."""
        if self.open and torch._C._current_graph_task_id() == -1:
            self._end()


REDUCE = _ReduceDefer()


def _deferred_reductions(backward):
    """Layer backward inside a deferred-reduction window (see _ReduceDefer)."""

    @functools.wraps(backward)
    def wrapped(ctx, *grads):
        flat = getattr(ctx, "flat", None)
        on = REDUCE.begin(getattr(flat, "device", None))
        try:
            return backward(ctx, *grads)
        finally:
            if on:
                REDUCE.pause()

    return wrapped


def _finish(flat: FlatParams, params, needs) -> None:
    done = [p for p, n in zip(params, needs) if n]
    for p in done:
        flat.attach(p)
    if done:
        if runtime._HOOKS:  # a hook (DDP bucket all-reduce) reads them: queued sums first
            REDUCE.flush()
        grads_ready(done)


def _wgrad(dy, x, out, **kw):
    """dW (+)= dy^T x on the weight-gradient stream (runtime.WGRAD). (Lone weight gradients as grouped
    launches of one measured slower: hybrid 6.52-6.61 -> 6.84-6.88 ms, an adapter's 6-tile gradient gets
    too few workgroups, profiles/r03af_single_wgrad_group_ab.txt.)"""
    return WGRAD.run(lambda: ops.linear_wgrad(dy, x, out, **kw), dy, x)


# Token counts up to which a layer's weight gradients go out as ONE grouped launch at the end of
# its backward (csrc/gemm.hip gemm_wgrad_group_kernel) instead of one split-K GEMM (+ reduction)
# each: the w+ latent (4,864 rows) and 48 px (640) configurations. ViT-B/16 (50,432 rows) keeps
# the per-weight split-K launches, issued as soon as each dY exists.
WGRAD_GROUP_MAX_M = 16384


class _WgradBatch:
    def __init__(self, M: int, dt: torch.dtype):
        self.on = dt == torch.bfloat16 and M <= WGRAD_GROUP_MAX_M
        self.items = []

    def add(self, dy, x, out, accumulate: bool) -> None:
        if out is None:
            return
        if self.on:
            self.items.append((dy, x, out, accumulate))
        else:
            _wgrad(dy, x, out, accumulate=accumulate)

    def flush(self) -> None:
        if self.items:
            items, self.items = self.items, []
            WGRAD.run(lambda: ops.linear_wgrad_group(items), *[t for it in items for t in it[:2]])


def _empty(M, N, like, dtype=None):
    return torch.empty(M, N, dtype=dtype or like.dtype, device=like.device)


# =========================================================== post-norm encoder layer
class PostNormLayerFn(torch.autograd.Function):
    # params: in_w, in_b, out_w, out_b, w1, b1, w2, b2, n1w, n1b, n2w, n2b
    @staticmethod
    def forward(ctx, x, cfg: LayerCfg, flat: FlatParams, *P):
        in_w, in_b, out_w, out_b, w1, b1, w2, b2, n1w, n1b, n2w, n2b = P
        M, D = x.shape
        F = w1.shape[0]
        dt = x.dtype
        dh = D // cfg.H
        pd = cfg.dropout
        seeds = [next_seed() for _ in range(4)] if pd > 0 else [0, 0, 0, 0]
        f32 = torch.float32
        qkv = ops.linear_fwd(x, _weight(flat, in_w, dt), in_b.data)
        o = _empty(M, D, x)
        lse = ops.attention_saved(qkv, cfg.B, cfg.N, cfg.H, dh, dropout=pd)
        ops.attention_fwd(qkv, o, lse, cfg.B, cfg.N, cfg.H, dh, dropout=pd, seed=seeds[0])
        y = ops.linear_fwd(o, _weight(flat, out_w, dt), out_b.data, res=x, dropout=pd, seed=seeds[1], drop_ld=D)
        m1 = torch.empty(M, dtype=f32, device=x.device)
        r1 = torch.empty_like(m1)
        x1 = ops.layernorm_fwd(y, n1w.data, n1b.data, cfg.eps, mean=m1, rstd=r1)
        f = _empty(M, F, x) if cfg.save else None
        # f = the backward gate act'(pre) * keep / (1 - p) of linear1's output: the linear2 dgrad
        # below applies GELU' and the dropout in one multiply
        g = ops.linear_fwd(x1, _weight(flat, w1, dt), b1.data, pre=f, pre_gate=True, act=cfg.act, dropout=pd,
                           seed=seeds[2], drop_ld=F)
        z = ops.linear_fwd(g, _weight(flat, w2, dt), b2.data, res=x1, dropout=pd, seed=seeds[3], drop_ld=D)
        m2 = torch.empty(M, dtype=f32, device=x.device)
        r2 = torch.empty_like(m2)
        out = ops.layernorm_fwd(z, n2w.data, n2b.data, cfg.eps, mean=m2, rstd=r2)
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P, ctx.seeds = cfg, flat, P, seeds
            ctx.saved = (x, qkv, o, lse, y, m1, r1, x1, f, g, z, m2, r2)
        return out

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dout):
        cfg, flat, P, seeds = ctx.cfg, ctx.flat, ctx.P, ctx.seeds
        in_w, in_b, out_w, out_b, w1, b1, w2, b2, n1w, n1b, n2w, n2b = P
        x, qkv, o, lse, y, m1, r1, x1, f, g, z, m2, r2 = ctx.saved
        needs = ctx.needs_input_grad[3:]
        G, acc = _targets(flat, P, needs)
        gin_w, gin_b, gout_w, gout_b, gw1, gb1, gw2, gb2, gn1w, gn1b, gn2w, gn2b = G
        dout = dout.contiguous()
        M, D = x.shape
        dt = x.dtype
        dh = D // cfg.H
        pd = cfg.dropout
        wb = _WgradBatch(M, dt)
        # LN2 (+ dropout of the FFN branch, + linear2 bias grad)
        dz = torch.empty_like(z)
        dh2 = torch.empty_like(z) if pd > 0 else None
        ops.layernorm_bwd(dout, z, m2, r2, n2w.data, dx=dz, dx_drop=dh2, dropout=pd, seed=seeds[3], dgamma=gn2w,
                          dbeta=gn2b, dbias=gb2, accumulate=acc)
        dh2 = dz if dh2 is None else dh2
        wb.add(dh2, g, gw2, acc)
        # linear1.bias grad = column sums of dF, fused into this GEMM's epilogue
        dF = _dgrad(flat, dh2, w2, dt, aux=f, aux_act="mul", colsum=gb1, colsum_accumulate=acc)
        wb.add(dF, x1, gw1, acc)
        dx1 = _dgrad(flat, dF, w1, dt, res=dz)
        # LN1 (+ dropout of the attention branch, + out_proj bias grad)
        dy = torch.empty_like(y)
        dhh = torch.empty_like(y) if pd > 0 else None
        ops.layernorm_bwd(dx1, y, m1, r1, n1w.data, dx=dy, dx_drop=dhh, dropout=pd, seed=seeds[1], dgamma=gn1w,
                          dbeta=gn1b, dbias=gout_b, accumulate=acc)
        dhh = dy if dhh is None else dhh
        wb.add(dhh, o, gout_w, acc)
        do = _dgrad(flat, dhh, out_w, dt)
        dqkv = _empty(M, 3 * D, x)
        ops.attention_bwd(qkv, o, do, lse, dqkv, cfg.B, cfg.N, cfg.H, dh, dropout=pd, seed=seeds[0], colsum=gin_b,
                          colsum_accumulate=acc)
        wb.add(dqkv, x, gin_w, acc)
        dx = _dgrad(flat, dqkv, in_w, dt, res=dy)
        wb.flush()
        _finish(flat, P, needs)
        ctx.saved = None
        return (dx, None, None) + (None,) * len(P)


# =========================================================== timm pre-norm block
class PreNormBlockFn(torch.autograd.Function):
    # params: n1w, n1b, qkv_w, qkv_b, proj_w, proj_b, n2w, n2b, fc1_w, fc1_b, fc2_w, fc2_b
    @staticmethod
    def forward(ctx, x, cfg: LayerCfg, flat: FlatParams, *P):
        n1w, n1b, qkv_w, qkv_b, proj_w, proj_b, n2w, n2b, fc1_w, fc1_b, fc2_w, fc2_b = P
        M, D = x.shape
        F = fc1_w.shape[0]
        dt = x.dtype
        dh = D // cfg.H
        f32 = torch.float32
        m1 = torch.empty(M, dtype=f32, device=x.device)
        r1 = torch.empty_like(m1)
        h1 = ops.layernorm_fwd(x, n1w.data, n1b.data, cfg.eps, mean=m1, rstd=r1)
        qkv = ops.linear_fwd(h1, _weight(flat, qkv_w, dt), qkv_b.data)
        o = _empty(M, D, x)
        lse = ops.attention_saved(qkv, cfg.B, cfg.N, cfg.H, dh)
        ops.attention_fwd(qkv, o, lse, cfg.B, cfg.N, cfg.H, dh)
        x2 = ops.linear_fwd(o, _weight(flat, proj_w, dt), proj_b.data, res=x)
        m2 = torch.empty(M, dtype=f32, device=x.device)
        r2 = torch.empty_like(m2)
        h2 = ops.layernorm_fwd(x2, n2w.data, n2b.data, cfg.eps, mean=m2, rstd=r2)
        f = _empty(M, F, x) if cfg.save else None
        g = ops.linear_fwd(h2, _weight(flat, fc1_w, dt), fc1_b.data, pre=f, pre_gate=True, act="gelu")
        out = ops.linear_fwd(g, _weight(flat, fc2_w, dt), fc2_b.data, res=x2)
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P = cfg, flat, P
            ctx.saved = (x, m1, r1, h1, qkv, o, lse, x2, m2, r2, h2, f, g)
        return out

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dout):
        cfg, flat, P = ctx.cfg, ctx.flat, ctx.P
        n1w, n1b, qkv_w, qkv_b, proj_w, proj_b, n2w, n2b, fc1_w, fc1_b, fc2_w, fc2_b = P
        x, m1, r1, h1, qkv, o, lse, x2, m2, r2, h2, f, g = ctx.saved
        needs = ctx.needs_input_grad[3:]
        G, acc = _targets(flat, P, needs)
        gn1w, gn1b, gqkv_w, gqkv_b, gproj_w, gproj_b, gn2w, gn2b, gfc1_w, gfc1_b, gfc2_w, gfc2_b = G
        dout = dout.contiguous()
        M, D = x.shape
        dt = x.dtype
        dh = D // cfg.H
        wb = _WgradBatch(M, dt)
        if gfc2_b is not None:
            ops.colsum(dout, gfc2_b, accumulate=acc)
        wb.add(dout, g, gfc2_w, acc)
        dF = _dgrad(flat, dout, fc2_w, dt, aux=f, aux_act="mul", colsum=gfc1_b, colsum_accumulate=acc)
        wb.add(dF, h2, gfc1_w, acc)
        dh2 = _dgrad(flat, dF, fc1_w, dt)
        dx2 = ops.layernorm_bwd(dh2, x2, m2, r2, n2w.data, res=dout, dgamma=gn2w, dbeta=gn2b, accumulate=acc)
        if gproj_b is not None:
            ops.colsum(dx2, gproj_b, accumulate=acc)
        wb.add(dx2, o, gproj_w, acc)
        do = _dgrad(flat, dx2, proj_w, dt)
        dqkv = _empty(M, 3 * D, x)
        ops.attention_bwd(qkv, o, do, lse, dqkv, cfg.B, cfg.N, cfg.H, dh, colsum=gqkv_b, colsum_accumulate=acc)
        wb.add(dqkv, h1, gqkv_w, acc)
        dh1 = _dgrad(flat, dqkv, qkv_w, dt)
        dx = ops.layernorm_bwd(dh1, x, m1, r1, n1w.data, res=dx2, dgamma=gn1w, dbeta=gn1b, accumulate=acc)
        wb.flush()
        _finish(flat, P, needs)
        ctx.saved = None
        return (dx, None, None) + (None,) * len(P)


# =========================================================== adapter
class AdapterFn(torch.autograd.Function):
    # params: fc1_w [A,D], fc1_b, fc2_w [D,A], fc2_b, alpha [1]
    @staticmethod
    def forward(ctx, x, cfg: LayerCfg, flat: FlatParams, *P):
        fc1_w, fc1_b, fc2_w, fc2_b, alpha = P
        M, D = x.shape
        A = fc1_w.shape[0]
        dt = x.dtype
        u = _empty(M, A, x) if cfg.save else None
        v = ops.linear_fwd(x, _weight(flat, fc1_w, dt), fc1_b.data, pre=u, pre_gate=True, act="gelu")
        T = _empty(M, D, x) if cfg.save else None
        out = ops.linear_fwd(v, _weight(flat, fc2_w, dt), fc2_b.data, pre=T, post_scale=alpha.data, res=x)
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P = cfg, flat, P
            ctx.saved = (x, u, v, T)
        return out

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dout):
        flat, P = ctx.flat, ctx.P
        fc1_w, fc1_b, fc2_w, fc2_b, alpha = P
        x, u, v, T = ctx.saved
        needs = ctx.needs_input_grad[3:]
        G, acc = _targets(flat, P, needs)
        g1w, g1b, g2w, g2b, galpha = G
        dout = dout.contiguous()
        dt = x.dtype
        a = alpha.data
        if galpha is not None:
            ops.dot(dout, T, galpha, accumulate=acc)
        if g2b is not None:
            ops.colsum(dout, g2b, accumulate=acc, scale=a)
        if g2w is not None:
            _wgrad(dout, v, g2w, accumulate=acc, post_scale=a)
        du = _dgrad(flat, dout, fc2_w, dt, post_scale=a, aux=u, aux_act="mul")
        if g1b is not None:
            ops.colsum(du, g1b, accumulate=acc)
        if g1w is not None:
            _wgrad(du, x, g1w, accumulate=acc)
        dx = _dgrad(flat, du, fc1_w, dt, res=dout)
        _finish(flat, P, needs)
        ctx.saved = None
        return (dx, None, None) + (None,) * len(P)


# =========================================================== embeddings
class PatchTokensFn(torch.autograd.Function):
    # params: proj_w [D,C,P,P], proj_b [D], cls [1,1,D], pos [1,N,D]
    @staticmethod
    def forward(ctx, img, cfg: LayerCfg, flat: FlatParams, dt: torch.dtype, patch: int, *P):
        proj_w, proj_b, cls, pos = P
        B = img.shape[0]
        D = proj_w.shape[0]
        img = img.contiguous().float()
        cols = ops.im2col_patch(img, patch, dt)
        Wm = _weight(flat, proj_w, dt).reshape(D, -1)
        emb = ops.linear_fwd(cols, Wm, proj_b.data)
        n = emb.shape[0] // B
        seed = next_seed() if cfg.dropout > 0 else 0
        t = ops.tokens_fwd(emb, cls.data, pos.data, B, n, D, dropout=cfg.dropout, seed=seed)
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P, ctx.seed, ctx.n = cfg, flat, P, seed, n
            ctx.saved = (cols,)
        return t

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dt_):
        cfg, flat, P = ctx.cfg, ctx.flat, ctx.P
        proj_w, proj_b, cls, pos = P
        (cols,) = ctx.saved
        needs = ctx.needs_input_grad[5:]
        G, acc = _targets(flat, P, needs)
        gw, gb, gcls, gpos = G
        D = proj_w.shape[0]
        demb = ops.tokens_bwd(dt_.contiguous(), cfg.B, ctx.n, D, gcls, gpos, acc, dropout=cfg.dropout,
                              seed=ctx.seed, want_demb=gw is not None or gb is not None)
        if gb is not None:
            ops.colsum(demb, gb, accumulate=acc)
        if gw is not None:
            _wgrad(demb, cols, gw.view(D, -1), accumulate=acc)
        _finish(flat, P, needs)
        ctx.saved = None
        return (None, None, None, None, None) + (None,) * len(P)


class LatentTokensFn(torch.autograd.Function):
    # params: in_w [E,Din], in_b [E], cls [1,1,E], pos [1,N,E]
    @staticmethod
    def forward(ctx, x, cfg: LayerCfg, flat: FlatParams, dt: torch.dtype, *P):
        in_w, in_b, cls, pos = P
        B, L, Din = x.shape
        E = in_w.shape[0]
        x2 = x.reshape(B * L, Din)
        xc = ops.cast_bf16(x2.contiguous().float()) if dt == torch.bfloat16 else x2.contiguous().float()
        emb = ops.linear_fwd(xc, _weight(flat, in_w, dt), in_b.data)
        t = ops.tokens_fwd(emb, cls.data, pos.data, B, L, E)
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P, ctx.L, ctx.xdtype = cfg, flat, P, L, x.dtype
            ctx.saved = (xc,)
        return t

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dt_):
        cfg, flat, P = ctx.cfg, ctx.flat, ctx.P
        in_w, in_b, cls, pos = P
        (xc,) = ctx.saved
        needs = ctx.needs_input_grad[4:]
        G, acc = _targets(flat, P, needs)
        gw, gb, gcls, gpos = G
        E = in_w.shape[0]
        B, L = cfg.B, ctx.L
        demb = ops.tokens_bwd(dt_.contiguous(), B, L, E, gcls, gpos, acc)
        if gb is not None:
            ops.colsum(demb, gb, accumulate=acc)
        if gw is not None:
            _wgrad(demb, xc, gw, accumulate=acc)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(B * L, xc.shape[1], dtype=torch.float32, device=xc.device)
            _dgrad(flat, demb, in_w, demb.dtype, out=dx)
            dx = dx.view(B, L, -1).to(ctx.xdtype)
        _finish(flat, P, needs)
        ctx.saved = None
        return (dx, None, None, None) + (None,) * len(P)


# =========================================================== head
class HeadFn(torch.autograd.Function):
    # params: ln_w, ln_b, W [C,D], b [C]
    @staticmethod
    def forward(ctx, t, cfg: LayerCfg, flat: FlatParams, *P):
        lnw, lnb, W, b = P
        seed = next_seed() if cfg.dropout > 0 else 0
        logits, stats = ops.head_fwd(t, cfg.N, lnw.data, lnb.data, cfg.eps, W.data, b.data, cfg.B,
                                     dropout=cfg.dropout, seed=seed)
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P, ctx.seed = cfg, flat, P, seed
            ctx.saved = (t, stats)
        return logits

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dlogits):
        cfg, flat, P = ctx.cfg, ctx.flat, ctx.P
        lnw, lnb, W, b = P
        t, stats = ctx.saved
        needs = ctx.needs_input_grad[3:]
        G, acc = _targets(flat, P, needs)
        dt = ops.head_bwd(t, cfg.N, lnw.data, lnb.data, W.data, stats, dlogits.contiguous().float(), cfg.B, G, acc,
                          dropout=cfg.dropout, seed=ctx.seed)
        _finish(flat, P, needs)
        ctx.saved = None
        return (dt, None, None) + (None,) * len(P)


# =========================================================== w+ prologue (fp32)
class WplusFn(torch.autograd.Function):
    """`spec` (modules/_wplus.py) maps the prologue's parameters to contiguous [L][D]
    views of the flat data / grad buffers; P lists the same parameters for autograd."""

    @staticmethod
    def forward(ctx, x, cfg: LayerCfg, flat: FlatParams, spec, *P):
        from ._lib import check, lib

        B, L, D = x.shape
        xc = x.contiguous().float()
        y = torch.empty_like(xc)
        saved = torch.empty(B * L * 2, dtype=torch.float32, device=x.device)
        sg, sl, lw, lb, gate, lm = spec.views(flat.data)
        check(lib().fer_wplus_fwd(xc.data_ptr(), y.data_ptr(), B, L, D, ops.ptr(sg), ops.ptr(sl),
                                  ops.ptr(spec.groups), ops.ptr(lw), ops.ptr(lb), ops.ptr(gate), ops.ptr(lm), 1e-5,
                                  saved.data_ptr(), ops.stream()), "wplus_fwd")
        if cfg.save:
            ctx.cfg, ctx.flat, ctx.P, ctx.spec = cfg, flat, P, spec
            ctx.saved = (xc, saved)
        return y

    @staticmethod
    @_deferred_reductions
    def backward(ctx, dy):
        from ._lib import check, lib

        flat, P, spec = ctx.flat, ctx.P, ctx.spec
        xc, saved = ctx.saved
        B, L, D = xc.shape
        needs = ctx.needs_input_grad[4:]
        _, acc = _targets(flat, P, needs)
        sg, sl, lw, lb, gate, lm = spec.views(flat.data)
        dsg, dsl, dlw, dlb, dgate, dlm = spec.views(flat.grad, needs=dict(zip(map(id, P), needs)))
        dyc = dy.contiguous().float()
        dx = torch.empty_like(xc)
        ws = ops.WS.get(lib().fer_wplus_ws(B, L, D), xc.device)
        check(lib().fer_wplus_bwd(xc.data_ptr(), saved.data_ptr(), dyc.data_ptr(), dx.data_ptr(), B, L, D,
                                  ops.ptr(sg), ops.ptr(sl), ops.ptr(spec.groups), ops.ptr(lw), ops.ptr(lb),
                                  ops.ptr(gate), ops.ptr(lm), 1e-5, ops.ptr(dsg), ops.ptr(dsl), ops.ptr(dlw),
                                  ops.ptr(dlb), ops.ptr(dgate), ops.ptr(dlm), int(acc), ws.data_ptr(),
                                  ws.numel() * 4, ops.stream()), "wplus_bwd")
        _finish(flat, P, needs)
        ctx.saved = None
        return (dx if ctx.needs_input_grad[0] else None, None, None, None) + (None,) * len(P)
