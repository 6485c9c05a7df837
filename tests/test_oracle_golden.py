"""Pin the CPU oracle (oracle/vit_oracle.py) to the reference's own outputs.

The fixtures were produced by running the reference model code
(`tests/golden/make_golden.py`); here the restatement must reproduce logits,
loss, every parameter gradient checksum and one AdamW step.
"""
import math

import numpy as np
import pytest
import torch

import vit_oracle as O
from cases import CASES, case_inputs, fixture_state_dict, load_fixture, oracle_forward
from detparams import det_directions, det_input


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_forward_backward_matches_reference(name):
    torch.set_num_threads(8)
    fx = load_fixture(name)
    p = {k: v.clone().requires_grad_(v.dtype.is_floating_point) for k, v in fixture_state_dict(fx).items()}
    x, y = case_inputs(name)
    logits = oracle_forward(name, x, p)
    np.testing.assert_allclose(logits.detach().numpy(), fx["logits"], atol=2e-5, rtol=1e-4)
    np.testing.assert_allclose(logits.detach().numpy(), fx["logits_eval"], atol=2e-5, rtol=1e-4)
    loss = O.cross_entropy(logits, y, label_smoothing=0.1)
    assert abs(loss.item() - float(fx["loss"])) < 1e-5
    loss.backward()
    for k, gs, gl2, samp, idx in zip(fx["grad_keys"], fx["grad_sum"], fx["grad_l2"], fx["grad_samples"],
                                     fx["grad_idx"]):
        g = p[str(k)].grad.reshape(-1).double()
        assert abs(g.norm().item() - gl2) <= 1e-4 * gl2 + 1e-7, k
        assert abs(g.sum().item() - gs) <= 1e-4 * (gl2 * math.sqrt(g.numel())) + 1e-6, k
        ok = idx >= 0
        np.testing.assert_allclose(g[idx[ok]].numpy(), samp[ok], atol=1e-6 + 1e-4 * gl2, err_msg=str(k))


@pytest.mark.parametrize("name", ["image_vit_48", "latent_vit_v2_all"])
def test_oracle_adamw_matches_reference(name):
    fx = load_fixture(name)
    p = {k: v.clone().requires_grad_(v.dtype.is_floating_point) for k, v in fixture_state_dict(fx).items()}
    x, y = case_inputs(name)
    O.cross_entropy(oracle_forward(name, x, p), y, label_smoothing=0.1).backward()
    for k, samp, idx, gsamp in zip(fx["grad_keys"], fx["adamw_samples"], fx["grad_idx"], fx["grad_samples"]):
        t = p[str(k)]
        wd = 0.05
        with torch.no_grad():
            m = torch.zeros_like(t)
            v = torch.zeros_like(t)
            O.adamw_step(t, t.grad, m, v, 1, 1e-3, wd=wd)
        # step 1 moves each weight by ~lr*sign(g): only well-conditioned where |g| >> eps
        ok = (idx >= 0) & (np.abs(np.nan_to_num(gsamp)) > 1e-5)
        np.testing.assert_allclose(t.detach().reshape(-1)[idx[ok]].double().numpy(), samp[ok], atol=2e-6)


def test_oracle_decomposer_matches_reference():
    fx = load_fixture("decomposer")
    dirs = O.normalize_directions(det_directions(7, 18, 512))
    assert abs(dirs.double().sum().item() - float(fx["directions_buffer_sum"])) < 1e-4
    w = det_input("decomposer", (4, 18, 512))
    for dm in ("all_classes", "max_class"):
        for om in ("expr_only", "id_only", "enhanced", "concat"):
            y = O.decomposer_forward(w, dirs, om, 2.0, dm).reshape(-1).double()
            assert tuple(fx[f"{dm}:{om}:shape"]) == tuple(O.decomposer_forward(w, dirs, om, 2.0, dm).shape)
            assert abs(y.norm().item() - float(fx[f"{dm}:{om}:l2"])) < 1e-3
            np.testing.assert_allclose(y[fx[f"{dm}:{om}:idx"]].numpy(), fx[f"{dm}:{om}:samples"], atol=1e-5)


def test_cross_entropy_class_weights_matches_torch():
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(16, 7, generator=g)
    y = torch.randint(0, 7, (16,), generator=g)
    w = torch.rand(7, generator=g) + 0.5
    for ls in (0.0, 0.1):
        ref = torch.nn.functional.cross_entropy(logits, y, weight=w, label_smoothing=ls)
        assert abs(O.cross_entropy(logits, y, ls, w).item() - ref.item()) < 1e-6


def test_oracle_adapter_matches_reference():
    """AdapterModule (`hybrid_latent_vit.py:249-265`) restated in the oracle == the reference's
    output and gradients on the committed fixture (cfg4 geometry 768 -> 64)."""
    from cases import adapter_inputs, check_summary

    fx = load_fixture("adapter")
    sd, x, dy = adapter_inputs()
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    x = x.clone().requires_grad_(True)
    y = O.adapter(x, p, "")
    (y * dy).sum().backward()
    check_summary(fx, "y", y, 1e-5)
    check_summary(fx, "dx", x.grad, 1e-5)
    for k in sd:
        check_summary(fx, "grad:" + k, p[k].grad, 1e-5)


def test_pos_embed_interpolation_matches_reference():
    """HybridLatentViT._init_position_embedding here == the reference's (`hybrid_latent_vit.py:
    118-156`) for seq_len 18 (w+), 36 (concat) and 196 (kept): same torch calls, bit-exact."""
    import types

    from cases import check_summary
    from models_fer_vit.hybrid_latent_vit import HybridLatentViT

    fx = load_fixture("pos_interp")
    pe = torch.nn.Parameter(det_input("pos_embed_vitb", (1, 197, 768)))
    stub = types.SimpleNamespace(pos_embed=pe)
    for L in (18, 36, 196):
        r = HybridLatentViT._init_position_embedding(types.SimpleNamespace(embed_dim=768), stub, L).detach()
        assert tuple(r.shape) == tuple(fx[f"L{L}:shape"])
        if L < 196:
            np.testing.assert_array_equal(r[0, :, :64].numpy(), fx[f"L{L}"])
        check_summary(fx, f"L{L}", r, 1e-7)
