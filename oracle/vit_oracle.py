"""CPU oracle for the FER-ViT training hot path — TEST INFRASTRUCTURE ONLY.

This module is a functional fp32 restatement, on the CPU, of the arithmetic the
reference (yuki-ominato/FER-ViT) runs on its hot path. Every function cites the
reference file:line it follows. It is imported only by `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg, and only as the
*checker* (or the timed CPU baseline); the product path in `fer-vit_amd/` never
imports it and fails loudly when its HIP library is missing.

Parity pinning: `tests/golden/make_golden.py` imports the reference's torch-only
model files (image_vit, latent_vit, latent_vit_v2, modules, latent_decomposer)
in the build container, runs them on deterministic weights/inputs and commits
the outputs under `tests/golden/`. `tests/test_oracle_golden.py` checks this
restatement against those fixtures. The timm pre-norm `Block` used by
HybridLatentViT / ExpressionAwareViT (timm 1.0.17, `environment.yml:124`) is not
vendored in the reference nor importable here, so `block_prenorm` is restated
from timm's published formula and is **parity unpinned**.

Written with explicit formulas (no nn.TransformerEncoderLayer / nn.MultiheadAttention),
so it is a restatement and not a call into the same module; backward comes from
torch autograd over these fp32 formulas (the reference's own backward is ATen
autograd too).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# `modules/semantic_pe.py:6-8`
LAYER_GROUPS = [0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2]


# --------------------------------------------------------------------------- ops
def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    """Row LayerNorm, biased variance (torch.nn.LayerNorm semantics)."""
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def gelu_erf(x: Tensor) -> Tensor:
    """Exact-erf GELU (`activation='gelu'`, `models_fer_vit/image_vit.py:106`)."""
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def patch_embed(x: Tensor, w: Tensor, b: Tensor, patch: int) -> Tensor:
    """Conv2d(k=P, s=P) as an im2col GEMM (`models_fer_vit/image_vit.py:27-44`).

    x [B,C,H,W] -> tokens [B, (H/P)*(W/P), D]; token n = row*(W/P)+col,
    K order (c, kh, kw) = the conv weight's [D, C, P, P] flattening.
    """
    B, C, H, W = x.shape
    gh, gw = H // patch, W // patch
    x = x[:, :, : gh * patch, : gw * patch]
    cols = x.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 1, 3, 5)
    cols = cols.reshape(B, gh * gw, C * patch * patch)
    return cols @ w.reshape(w.shape[0], -1).t() + b


def attention(q: Tensor, k: Tensor, v: Tensor, p_drop: float = 0.0) -> Tensor:
    """softmax(q k^T / sqrt(dh)) [dropout] v per (batch, head); q,k,v [B,H,N,dh]."""
    dh = q.shape[-1]
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    p = torch.softmax(s, dim=-1)
    if p_drop > 0:
        p = F.dropout(p, p_drop)
    return p @ v


def mha(x: Tensor, w_in: Tensor, b_in: Tensor, w_out: Tensor, b_out: Tensor, heads: int,
        p_drop: float = 0.0) -> Tensor:
    """nn.MultiheadAttention self-attention with packed in_proj (rows q|k|v),
    as used by nn.TransformerEncoderLayer (`image_vit.py:101`, `latent_vit.py:24`)."""
    B, N, D = x.shape
    dh = D // heads
    qkv = x @ w_in.t() + b_in
    q, k, v = qkv.split(D, dim=-1)
    sh = lambda t: t.reshape(B, N, heads, dh).permute(0, 2, 1, 3)
    o = attention(sh(q), sh(k), sh(v), p_drop).permute(0, 2, 1, 3).reshape(B, N, D)
    return o @ w_out.t() + b_out


def encoder_layer_postnorm(x: Tensor, p: Dict[str, Tensor], prefix: str, heads: int,
                           act: str, eps: float = 1e-5, p_drop: float = 0.0) -> Tensor:
    """nn.TransformerEncoderLayer(norm_first=False):
    x = LN1(x + Drop(SA(x))); x = LN2(x + Drop(W2 Drop(act(W1 x + b1)) + b2)),
    attention-probability dropout inside SA. GELU-erf for ImageViT (`image_vit.py:101-109`),
    ReLU default for LatentViT (`latent_vit.py:24-30`). Parity uses p_drop = 0."""
    g = lambda n: p[prefix + n]
    d = (lambda t: F.dropout(t, p_drop)) if p_drop > 0 else (lambda t: t)
    sa = mha(x, g("self_attn.in_proj_weight"), g("self_attn.in_proj_bias"),
             g("self_attn.out_proj.weight"), g("self_attn.out_proj.bias"), heads, p_drop)
    x = layer_norm(x + d(sa), g("norm1.weight"), g("norm1.bias"), eps)
    h = x @ g("linear1.weight").t() + g("linear1.bias")
    h = d(gelu_erf(h) if act == "gelu" else torch.relu(h))
    ff = h @ g("linear2.weight").t() + g("linear2.bias")
    return layer_norm(x + d(ff), g("norm2.weight"), g("norm2.bias"), eps)


def block_prenorm(x: Tensor, p: Dict[str, Tensor], prefix: str, heads: int, eps: float = 1e-6) -> Tensor:
    """timm 1.0.17 `vision_transformer.Block` (used at `hybrid_latent_vit.py:227-233`):
    x = x + attn(LN1(x)); x = x + fc2(GELU(fc1(LN2(x)))); qkv bias, no layer-scale,
    no dropout. PARITY UNPINNED (timm absent from the reference and this image)."""
    g = lambda n: p[prefix + n]
    h = layer_norm(x, g("norm1.weight"), g("norm1.bias"), eps)
    x = x + mha(h, g("attn.qkv.weight"), g("attn.qkv.bias"), g("attn.proj.weight"), g("attn.proj.bias"), heads)
    h = layer_norm(x, g("norm2.weight"), g("norm2.bias"), eps)
    h = gelu_erf(h @ g("mlp.fc1.weight").t() + g("mlp.fc1.bias"))
    return x + h @ g("mlp.fc2.weight").t() + g("mlp.fc2.bias")


def adapter(x: Tensor, p: Dict[str, Tensor], prefix: str) -> Tensor:
    """AdapterModule: x + alpha * fc2(GELU(fc1 x)) (`hybrid_latent_vit.py:249-265`)."""
    g = lambda n: p[prefix + n]
    h = gelu_erf(x @ g("adapter.0.weight").t() + g("adapter.0.bias"))
    return x + g("alpha") * (h @ g("adapter.2.weight").t() + g("adapter.2.bias"))


def leam(x: Tensor, w: Tensor) -> Tensor:
    """LEAM: x * sigmoid(w)[l] (`modules/leam.py:31-40`)."""
    return x * torch.sigmoid(w)[None, :, None]


def semantic_pe(x: Tensor, group_embed: Tensor, layer_embed: Tensor, groups: Tensor) -> Tensor:
    """SemanticPE: x + group_embed[groups[l]] + layer_embed[l] (`modules/semantic_pe.py:36-48`)."""
    L = x.shape[1]
    return x + (group_embed[groups.long()] + layer_embed[:L])[None]


def layer_wise_norm(x: Tensor, w: Tensor, b: Tensor, gate: Optional[Tensor], eps: float = 1e-5) -> Tensor:
    """LayerWiseNorm: per-token-index LN (w,b [L,D]); optional residual gate
    x + sigmoid(gate[l]) * (LN_l(x) - x) (`modules/layer_wise_norm.py:35-50`)."""
    n = layer_norm(x, w[None], b[None], eps)
    if gate is None:
        return n
    s = torch.sigmoid(gate)[None, :, None]
    return x + s * (n - x)


def decompose(w_plus: Tensor, dirs: Tensor, mode: str = "all_classes"):
    """LatentDecomposer.decompose (`models_fer_vit/latent_decomposer.py:82-119`);
    dirs [C, L, D] already renormalised (`:57-63`)."""
    B = w_plus.shape[0]
    C = dirs.shape[0]
    df = dirs.reshape(C, -1)
    wf = w_plus.reshape(B, -1)
    coeff = wf @ df.t()
    if mode == "all_classes":
        ef = coeff @ df
    elif mode == "max_class":
        best = coeff.abs().argmax(dim=1)
        ef = coeff[torch.arange(B), best][:, None] * df[best]
    else:
        raise ValueError(mode)
    w_expr = ef.reshape(w_plus.shape)
    return w_expr, w_plus - w_expr


def decomposer_forward(w_plus: Tensor, dirs: Tensor, output_mode: str = "expr_only",
                       enhance_alpha: float = 2.0, decompose_mode: str = "all_classes") -> Tensor:
    """LatentDecomposer.forward (`latent_decomposer.py:121-173`)."""
    e, i = decompose(w_plus, dirs, decompose_mode)
    if output_mode == "expr_only":
        return e
    if output_mode == "id_only":
        return i
    if output_mode == "enhanced":
        return i + enhance_alpha * e
    if output_mode == "concat":
        return torch.cat([e, i], dim=1)
    raise ValueError(output_mode)


def normalize_directions(dirs: Tensor) -> Tensor:
    """`latent_decomposer.py:57-63`: each class direction scaled to unit L2 norm (+1e-12)."""
    C = dirs.shape[0]
    f = dirs.reshape(C, -1)
    return (f / (f.norm(dim=1, keepdim=True) + 1e-12)).reshape(dirs.shape)


def cross_entropy(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0,
                  weight: Optional[Tensor] = None) -> Tensor:
    """nn.CrossEntropyLoss(label_smoothing, weight), mean reduction
    (`train/train_image_vit.py:262-267`), written out: with log-probs lp,
    loss_i = w[y_i] (1-eps) (-lp[y_i]) + eps/C sum_c w[c] (-lp[c]);
    normalised by sum_i w[y_i] (torch semantics)."""
    C = logits.shape[1]
    lp = torch.log_softmax(logits, dim=1)
    w = torch.ones(C, dtype=logits.dtype) if weight is None else weight
    nll = -lp.gather(1, labels[:, None])[:, 0] * w[labels]
    smooth = -(lp * w[None]).sum(1)
    denom = w[labels].sum()
    return ((1 - label_smoothing) * nll.sum() + label_smoothing / C * smooth.sum()) / denom


# ------------------------------------------------------------------------ models
def image_vit_forward(x: Tensor, p: Dict[str, Tensor], patch: int, heads: int, depth: int,
                      p_drop: float = 0.0) -> Tensor:
    """ImageViT.forward (`models_fer_vit/image_vit.py:138-166`)."""
    B = x.shape[0]
    t = patch_embed(x, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"], patch)
    t = torch.cat([p["cls_token"].expand(B, -1, -1), t], 1) + p["pos_embed"]
    if p_drop > 0:
        t = F.dropout(t, p_drop)
    for i in range(depth):
        t = encoder_layer_postnorm(t, p, f"transformer.layers.{i}.", heads, "gelu", p_drop=p_drop)
    c = layer_norm(t[:, 0], p["norm.weight"], p["norm.bias"], 1e-5)
    return c @ p["head.weight"].t() + p["head.bias"]


def latent_vit_forward(x: Tensor, p: Dict[str, Tensor], heads: int, depth: int, prefix: str = "") -> Tensor:
    """LatentViT.forward (`models_fer_vit/latent_vit.py:38-48`), ReLU post-norm layers."""
    g = lambda n: p[prefix + n]
    B = x.shape[0]
    t = x @ g("input_proj.weight").t() + g("input_proj.bias")
    t = torch.cat([g("cls_token").expand(B, -1, -1), t], 1) + g("pos_emb")
    for i in range(depth):
        t = encoder_layer_postnorm(t, p, f"{prefix}transformer.layers.{i}.", heads, "relu")
    c = layer_norm(t[:, 0], g("mlp_head.0.weight"), g("mlp_head.0.bias"), 1e-5)
    return c @ g("mlp_head.1.weight").t() + g("mlp_head.1.bias")


def wplus_prologue(x: Tensor, p: Dict[str, Tensor], use_spe: bool, use_lwn: bool,
                   use_lwn_residual: bool, use_leam: bool) -> Tensor:
    """LatentViTv2 prologue order SPE -> LWN -> LEAM (`models_fer_vit/latent_vit_v2.py:82-84`)."""
    L = x.shape[1]
    if use_spe:
        x = semantic_pe(x, p["spe.group_embed.weight"], p["spe.layer_embed.weight"], p["spe.groups"])
    if use_lwn:
        w = torch.stack([p[f"lwn.norms.{i}.weight"] for i in range(L)])
        b = torch.stack([p[f"lwn.norms.{i}.bias"] for i in range(L)])
        x = layer_wise_norm(x, w, b, p["lwn.gate"] if use_lwn_residual else None)
    if use_leam:
        x = leam(x, p["leam.layer_weights"])
    return x


def latent_vit_v2_forward(x: Tensor, p: Dict[str, Tensor], heads: int, depth: int, use_spe: bool,
                          use_lwn: bool, use_lwn_residual: bool, use_leam: bool) -> Tensor:
    """LatentViTv2.forward (`models_fer_vit/latent_vit_v2.py:75-85`)."""
    x = wplus_prologue(x, p, use_spe, use_lwn, use_lwn_residual, use_leam)
    return latent_vit_forward(x, p, heads, depth, prefix="backbone.")


def hybrid_forward(x: Tensor, p: Dict[str, Tensor], heads: int, depth: int, use_adapter: bool,
                   prefix: str = "") -> Tensor:
    """HybridLatentViT.forward (`models_fer_vit/hybrid_latent_vit.py:205-239`); head =
    LN(1e-5) -> Dropout(off) -> Linear (`:110-114`)."""
    g = lambda n: p[prefix + n]
    B = x.shape[0]
    t = x @ g("input_proj.weight").t() + g("input_proj.bias")
    t = torch.cat([g("cls_token").expand(B, -1, -1), t], 1) + g("pos_embed")
    for i in range(depth):
        t = block_prenorm(t, p, f"{prefix}transformer.{i}.", heads)
        if use_adapter:
            t = adapter(t, p, f"{prefix}adapters.{i}.")
    c = layer_norm(t[:, 0], g("head.0.weight"), g("head.0.bias"), 1e-5)
    return c @ g("head.2.weight").t() + g("head.2.bias")


def adamw_step(param: Tensor, grad: Tensor, m: Tensor, v: Tensor, step: int, lr: float,
               beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8, wd: float = 0.0):
    """torch.optim.AdamW single-tensor update (decoupled weight decay), in place;
    the optimizer the trainers build (`train/train_image_vit.py:270-276`)."""
    param.mul_(1 - lr * wd)
    m.mul_(beta1).add_(grad, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(m, denom, value=-lr / bc1)
