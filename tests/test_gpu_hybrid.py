"""HybridLatentViT / ExpressionAwareViT on the GPU against the oracle restatement.

timm's Block is absent from the reference and this image, so the whole models are
PARITY UNPINNED against the reference (their timm-free pieces are pinned: AdapterModule and the
LatentDecomposer against reference-generated fixtures below, the 196 -> L pos-embed interpolation
in tests/test_oracle_golden.py); they are checked against `oracle.hybrid_forward`
(timm 1.0.17 pre-norm Block formula, `hybrid_latent_vit.py:205-265`) with torch autograd
through the oracle for the gradients. Eval mode (the head dropout is the only dropout).
Tolerances: fp32 path logits 1e-3, per-parameter gradient L2 within 2e-3 relative; bf16 path per-test
gates at 2x the measured errors (BF16_GATES).
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


def _oracle(m, x, y, use_adapter, decomposer=None, heads=3, output_mode="expr_only", decompose_mode="all_classes",
            spe=False, leam=False):
    p = {k: v.detach().float().clone().requires_grad_(v.dtype.is_floating_point)
         for k, v in m.state_dict().items()}
    prefix = ""
    if decomposer is not None:
        prefix = "vit."
        x = O.decomposer_forward(x, O.normalize_directions(decomposer), output_mode, 2.0, decompose_mode)
        x = O.wplus_prologue(x, p, spe, False, False, leam)
    logits = O.hybrid_forward(x, p, heads=heads, depth=12, use_adapter=use_adapter, prefix=prefix)
    loss = O.cross_entropy(logits, y, label_smoothing=0.1)
    loss.backward()
    return logits.detach(), {k: v.grad for k, v in p.items() if v.grad is not None}


# bf16 gates per test, at 2x the errors measured on the GPU (tests/bf16_parity_measure.py --hybrid,
# profiles/r05*_bf16_parity_hybrid.json): (max |logits - ref| / max(1, max |ref|), per-parameter gradient
# L2 error / ||ref|| over the non-scalar parameters, the same for the scalar adapter alphas). The alphas'
# gradients are near-cancelling sums over B*N*D terms (test_adapter_matches_reference_fixture
# quantifies that), hence their own, wider gate.
# Measured (r05a, MI355X): hybrid_adapter 0.0114 / 0.0111 / 0.0166, cfg4 0.0069 / 0.0173 / 0.171, cfg5
# 0.0082 / 0.0160 / 0.173. (The cfg4 / cfg5 alphas: 12 scalars whose gradients cancel to ~1e-3 of their
# terms' magnitude; every other trainable gradient is within 1.8 %.)
BF16_GATES = {
    "hybrid_adapter": (0.023, 0.022, 0.034),
    "cfg4": (0.014, 0.035, 0.35),
    "cfg5": (0.017, 0.032, 0.35),
}


def _errors(m, x, y, ref_logits, ref_grads, prec, frozen_prefix=None):
    """(logit error / max(1, max|ref|), max gradient rel L2 error, max scalar-gradient rel error, #checked)"""
    m.set_precision(prec).eval()
    logits = m(x.cuda())
    torch.nn.functional.cross_entropy(logits, y.cuda(), label_smoothing=0.1).backward()
    lg = logits.detach().float().cpu()
    lerr = (lg - ref_logits).abs().max().item() / max(1.0, ref_logits.abs().max().item())
    gerr, serr, n_checked = 0.0, 0.0, 0
    for k, p in m.named_parameters():
        if frozen_prefix and k.startswith(frozen_prefix):
            assert p.grad is None or not p.requires_grad, k
            continue
        if not p.requires_grad:
            continue
        r = ref_grads[k]
        g = p.grad.detach().float().cpu()
        e = (g - r).norm().item() / (r.norm().item() + 1e-6)
        if p.numel() == 1:
            serr = max(serr, e)
        else:
            gerr = max(gerr, e)
        n_checked += 1
    return lerr, gerr, serr, n_checked


def _check(m, x, y, ref_logits, ref_grads, prec, frozen_prefix=None, gate="hybrid_adapter"):
    lerr, gerr, serr, n_checked = _errors(m, x, y, ref_logits, ref_grads, prec, frozen_prefix)
    if prec == "fp32":
        ltol, gtol, stol = 1e-3, 2e-3, 2e-3
    else:
        ltol, gtol, stol = BF16_GATES[gate]
    assert lerr < ltol, (lerr, ltol)
    assert gerr <= gtol, (gerr, gtol)
    assert serr <= stol, (serr, stol)
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


# ------------------------------------------------------------------ reference-pinned pieces
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_adapter_matches_reference_fixture(prec):
    """fervit AdapterModule (HIP: fc1 + GELU epilogue, fc2 + alpha-residual epilogue) against
    the REFERENCE AdapterModule's output and gradients (`hybrid_latent_vit.py:249-265`,
    tests/golden/adapter.npz) at the cfg4 geometry 768 -> 64 -> 768."""
    from cases import adapter_inputs, check_summary, load_fixture
    from fervit.blocks import AdapterModule

    fx = load_fixture("adapter")
    sd, x, dy = adapter_inputs()
    m = AdapterModule(768, 64)
    m.load_state_dict(sd)
    m = m.cuda().set_precision(prec)
    xg = x.cuda().requires_grad_(True)
    out = m(xg)
    (out.float() * dy.cuda()).sum().backward()
    rel = 1e-4 if prec == "fp32" else 2e-2
    check_summary(fx, "y", out.float(), rel)
    check_summary(fx, "dx", xg.grad, rel)
    params = dict(m.named_parameters())
    for k in sd:
        if k == "alpha" and prec == "bf16":
            # d alpha = sum(dy * a) over 58k terms that nearly cancel (|sum| ~ 2 vs sum|dy a| ~ 2e4):
            # with dy and a rounded to bf16 (2^-9 relative each) the expected error is
            # ~2^-9 * ||dy o a||, so the bound is stated against that scale (fp32: 1e-4 rel above)
            import vit_oracle as O

            a = O.adapter(x, sd, "") - x
            scale = (dy * a / 0.37).norm().item()
            err = abs(params[k].grad.item() - float(fx["grad:alpha:sum"]))
            assert err <= 4 * 2 ** -8 * scale, (err, scale)
            continue
        check_summary(fx, "grad:" + k, params[k].grad, rel if prec == "fp32" else 4e-2)


def test_decomposer_all_modes_match_reference():
    """fer_decompose in all 8 (decompose_mode, output_mode) combinations, including the
    concat route's [B, 36, 512] output, and the expression scores, against the REFERENCE
    LatentDecomposer's outputs (`latent_decomposer.py:82-173`, tests/golden/decomposer.npz)."""
    from cases import load_fixture
    from detparams import det_input
    from models_fer_vit.latent_decomposer import LatentDecomposer

    fx = load_fixture("decomposer")
    dirs = det_directions(7, 18, 512)
    dec = LatentDecomposer({i: dirs[i] for i in range(7)}, 18, 512).cuda()
    assert abs(dec.directions.double().sum().item() - float(fx["directions_buffer_sum"])) < 1e-4
    w = det_input("decomposer", (4, 18, 512)).cuda()
    for dm in ("all_classes", "max_class"):
        for om in ("expr_only", "id_only", "enhanced", "concat"):
            y = dec(w, output_mode=om, enhance_alpha=2.0, decompose_mode=dm)
            assert tuple(y.shape) == tuple(fx[f"{dm}:{om}:shape"]), (dm, om)
            yf = y.reshape(-1).double().cpu()
            assert abs(yf.norm().item() - float(fx[f"{dm}:{om}:l2"])) < 1e-4 * float(fx[f"{dm}:{om}:l2"]), (dm, om)
            np.testing.assert_allclose(yf[fx[f"{dm}:{om}:idx"]].numpy(), fx[f"{dm}:{om}:samples"], atol=2e-5,
                                       err_msg=f"{dm}:{om}")
        if dm == "all_classes":
            np.testing.assert_allclose(dec.get_expression_scores(w).cpu().numpy(), fx[f"{dm}:scores"], atol=1e-4)


# ------------------------------------------------------------------ BASELINE cfg4 / cfg5 geometry
def _perturb(m, seed):
    with torch.no_grad():
        g = torch.Generator().manual_seed(seed)
        for n, p in m.named_parameters():
            if n.endswith("alpha"):
                p.fill_(0.37)
            elif n.endswith("layer_weights"):
                p.add_(0.3 * torch.randn(p.shape, generator=g))
            elif p.dim() == 1 or "norm" in n or "head.0" in n:
                p.add_(0.1 * torch.randn(p.shape, generator=g))
            elif "adapters" in n:
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
    return m


def _hybrid_base(seq_len=18):
    """BASELINE cfg4: create_hybrid_latent_vit(model_size='base', use_pretrained=False,
    freeze_transformer=True, use_adapter=True, adapter_dim=64) on w+ latents (512)."""
    from models_fer_vit.hybrid_latent_vit import create_hybrid_latent_vit

    torch.manual_seed(4)
    return create_hybrid_latent_vit(latent_dim=512, seq_len=seq_len, model_size="base", use_pretrained=False,
                                    freeze_transformer=True, use_adapter=True, adapter_dim=64)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_cfg4_hybrid_base_frozen_adapter_matches_oracle(prec):
    """cfg4 geometry: timm ViT-B/16 blocks (D 768, 12 heads, 12 blocks, MLP 3072) frozen, adapters
    of width 64, w+ 512 input, B=4 -- logits and every trainable gradient vs the oracle."""
    m = _perturb(_hybrid_base(), 21)
    g = torch.Generator().manual_seed(9)
    x, y = torch.randn(4, 18, 512, generator=g), torch.randint(0, 7, (4,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=True, heads=12)
    _check(m.cuda(), x, y, ref_logits, ref_grads, prec, frozen_prefix="transformer.", gate="cfg4")


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_cfg5_expression_spe_leam_hybrid_base_matches_oracle(prec):
    """cfg5 composition: decomposer (7 unit directions, all_classes, expr_only) -> SPE -> LEAM
    -> the cfg4 hybrid (build-defined order), B=4, vs the oracle."""
    from models_fer_vit.expression_aware_vit import ExpressionAwareViT
    from models_fer_vit.latent_decomposer import LatentDecomposer

    dirs = det_directions(7, 18, 512)
    dec = LatentDecomposer({i: dirs[i] for i in range(7)})
    torch.manual_seed(5)
    m = _perturb(ExpressionAwareViT(dec, _hybrid_base(), output_mode="expr_only", decompose_mode="all_classes",
                                    use_spe=True, use_leam=True), 22)
    g = torch.Generator().manual_seed(10)
    x, y = torch.randn(4, 18, 512, generator=g), torch.randint(0, 7, (4,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=True, decomposer=dirs, heads=12, spe=True, leam=True)
    _check(m.cuda(), x, y, ref_logits, ref_grads, prec, frozen_prefix="vit.transformer.", gate="cfg5")


@pytest.mark.parametrize("decompose_mode", ["all_classes", "max_class"])
def test_expression_concat_route_matches_oracle(decompose_mode):
    """output_mode='concat' doubles the sequence (`expression_aware_vit.py:87`): 36 w+ tokens +
    CLS = 37-token attention, positional embedding interpolated 196 -> 36."""
    from models_fer_vit.expression_aware_vit import ExpressionAwareViT
    from models_fer_vit.hybrid_latent_vit import HybridLatentViT
    from models_fer_vit.latent_decomposer import LatentDecomposer

    dirs = det_directions(7, L, LAT)
    dec = LatentDecomposer({i: dirs[i] for i in range(7)}, seq_len=L, latent_dim=LAT)
    torch.manual_seed(3)
    vit = HybridLatentViT(latent_dim=LAT, seq_len=2 * L, pretrained_model_name="vit_tiny_patch16_224",
                          use_pretrained=False, adapter_dim=32)
    m = _perturb(ExpressionAwareViT(dec, vit, output_mode="concat", decompose_mode=decompose_mode), 23)
    g = torch.Generator().manual_seed(12)
    x, y = torch.randn(B, L, LAT, generator=g), torch.randint(0, 7, (B,), generator=g)
    ref_logits, ref_grads = _oracle(m, x, y, use_adapter=True, decomposer=dirs, output_mode="concat",
                                    decompose_mode=decompose_mode)
    _check(m.cuda(), x, y, ref_logits, ref_grads, "fp32")


def test_cfg4_bs256_bf16_matches_fp32_path():
    """cfg4 at its bench batch (bs 256, w+ 18 x 512): the bf16 production path against this library's
    fp32 parity path on identical weights and inputs (eval) -- logits within the gate and argmax equal
    on every sample whose fp32 top-2 margin exceeds 0.2."""
    m = _perturb(_hybrid_base(), 24).cuda()
    g = torch.Generator().manual_seed(13)
    x = torch.randn(256, 18, 512, generator=g).cuda()
    out = {}
    with torch.no_grad():
        for prec in ("fp32", "bf16"):
            m.set_precision(prec).eval()
            out[prec] = m(x).float().cpu()
    a, b = out["fp32"], out["bf16"]
    err = (a - b).abs().max().item() / max(1.0, a.abs().max().item())
    assert err < BF16_GATES_BS256["cfg4_bs256"], err
    top2 = a.topk(2, dim=1).values
    sure = (top2[:, 0] - top2[:, 1]) > 0.2
    assert sure.sum().item() > 0
    assert (a.argmax(1)[sure] == b.argmax(1)[sure]).all()


BF16_GATES_BS256 = {"cfg4_bs256": 0.023}  # 2x the measured 0.0112 (r05a; argmax equal on all 223 sure samples)
