"""HybridLatentViT / ExpressionAwareViT on the GPU against the oracle restatement.

timm's Block is absent from the reference and this image, so these models are
PARITY UNPINNED against the reference; they are checked against `oracle.hybrid_forward`
(timm 1.0.17 pre-norm Block formula, `hybrid_latent_vit.py:205-265`) with torch autograd
through the oracle for the gradients. Eval mode (the head dropout is the only dropout).
Tolerances: fp32 path logits 1e-3, per-parameter gradient L2 within 2e-3 relative.
"""
import numpy as np
import pytest
import torch

import vit_oracle as O
from detparams import det_directions

pytestmark = pytest.mark.gpu

B, L, LAT = 6, 18, 64


def _hybrid(adapter_dim=32, **kw):
    from models_fer_vit.hybrid_latent_vit import HybridLatentViT

    torch.manual_seed(3)
    m = HybridLatentViT(latent_dim=LAT, seq_len=L, pretrained_model_name="vit_tiny_patch16_224", num_classes=7,
                        use_pretrained=False, adapter_dim=adapter_dim, **kw)
    with torch.no_grad():  # move off the trivial init so every path carries signal
        g = torch.Generator().manual_seed(11)
        for n, p in m.named_parameters():
            if n.endswith("alpha"):
                p.fill_(0.37)
            elif p.dim() == 1 or "norm" in n or "head.0" in n:
                p.add_(0.1 * torch.randn(p.shape, generator=g))
            elif n.startswith("adapters"):
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
    return m


def _oracle(m, x, y, use_adapter, decomposer=None):
    p = {k: v.detach().float().clone().requires_grad_(v.dtype.is_floating_point)
         for k, v in m.state_dict().items()}
    prefix = ""
    if decomposer is not None:
        prefix = "vit."
        x = O.decomposer_forward(x, O.normalize_directions(decomposer), "expr_only")
    logits = O.hybrid_forward(x, p, heads=3, depth=12, use_adapter=use_adapter, prefix=prefix)
    loss = O.cross_entropy(logits, y, label_smoothing=0.1)
    loss.backward()
    return logits.detach(), {k: v.grad for k, v in p.items() if v.grad is not None}


def _check(m, x, y, ref_logits, ref_grads, prec, frozen_prefix=None):
    m.set_precision(prec).eval()
    logits = m(x.cuda())
    torch.nn.functional.cross_entropy(logits, y.cuda(), label_smoothing=0.1).backward()
    lg = logits.detach().cpu()
    tol = 1e-3 if prec == "fp32" else 5e-2 * max(1.0, ref_logits.abs().max().item())
    assert (lg - ref_logits).abs().max().item() < tol
    gtol = 2e-3 if prec == "fp32" else 8e-2
    n_checked = 0
    for k, p in m.named_parameters():
        if frozen_prefix and k.startswith(frozen_prefix):
            assert p.grad is None or not p.requires_grad, k
            continue
        if not p.requires_grad:
            continue
        r = ref_grads[k]
        g = p.grad.detach().float().cpu()
        rn = r.norm().item()
        assert (g - r).norm().item() <= gtol * rn + 1e-6, (k, (g - r).norm().item(), rn)
        n_checked += 1
    assert n_checked > 0


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_hybrid_adapter_matches_oracle(prec):
    m = _hybrid()
    g = torch.Generator().manual_seed(5)
    x, y = torch.randn(B, L, LAT, generator=g), torch.randint(0, 7, (B,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=True)
    _check(m.cuda(), x, y, ref_logits, ref_grads, prec)


def test_hybrid_frozen_transformer_adapter_strategy():
    m = _hybrid(freeze_transformer=True)
    g = torch.Generator().manual_seed(6)
    x, y = torch.randn(B, L, LAT, generator=g), torch.randint(0, 7, (B,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=True)
    _check(m.cuda(), x, y, ref_logits, ref_grads, "fp32", frozen_prefix="transformer.")


def test_hybrid_no_adapter_full_finetune():
    m = _hybrid(adapter_dim=None)
    g = torch.Generator().manual_seed(7)
    x, y = torch.randn(B, L, LAT, generator=g), torch.randint(0, 7, (B,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=False)
    _check(m.cuda(), x, y, ref_logits, ref_grads, "fp32")


def test_expression_aware_vit_matches_oracle():
    from models_fer_vit.expression_aware_vit import ExpressionAwareViT
    from models_fer_vit.latent_decomposer import LatentDecomposer

    dirs = det_directions(7, L, LAT)
    dec = LatentDecomposer({i: dirs[i] for i in range(7)}, seq_len=L, latent_dim=LAT)
    m = ExpressionAwareViT(dec, _hybrid())
    g = torch.Generator().manual_seed(8)
    x, y = torch.randn(B, L, LAT, generator=g), torch.randint(0, 7, (B,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=True, decomposer=dirs)
    _check(m.cuda(), x, y, ref_logits, ref_grads, "fp32")
