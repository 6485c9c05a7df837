"""The trainers' step functions (fer-vit_amd/train, `train/train_*.py` train_epoch / evaluate)
on the MI355X modules: the step sequence equals a hand-written loop of the reference's step
(same host RNG use for mixup, so identical batches and losses), metrics match sklearn on the
same predictions, and training decreases the loss."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _loader(n, shape, seed, bs):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, *shape, generator=g)
    y = torch.randint(0, 7, (n,), generator=g)
    ds = torch.utils.data.TensorDataset(x, y)
    return torch.utils.data.DataLoader(ds, batch_size=bs, shuffle=False)


def _latent_model(seed=0):
    from models_fer_vit.latent_vit_v2 import LatentViTv2

    torch.manual_seed(seed)
    return LatentViTv2(embed_dim=128, depth=2, heads=4, mlp_dim=256, dropout=0.0, use_lwn=True, use_spe=True,
                       use_leam=True).to(DEV)


def test_latent_v2_epoch_matches_reference_loop():
    """train_epoch (fused clip + FusedAdamW, device-side metrics) == the reference's loop body
    (`train/train_latent_vit_v2.py:114-141`) written with torch.nn.utils.clip_grad_norm_ and
    torch.optim.AdamW, per-step syncs included. fp32 compute path, so the only difference is
    the optimizer arithmetic (fused kernel vs torch's foreach AdamW)."""
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from train.train_latent_vit_v2 import evaluate, train_epoch

    loader = _loader(96, (18, 512), 1, 32)
    args = types.SimpleNamespace(mixup=1.0, grad_clip=1.0)
    crit = CrossEntropyLoss(label_smoothing=0.1)
    # ours
    m1 = _latent_model().set_precision("fp32")
    o1 = FusedAdamW(m1.parameters(), lr=1e-3, weight_decay=0.05, model=m1)
    np.random.seed(3)
    torch.manual_seed(3)
    loss1, acc1, f1_1 = train_epoch(m1, loader, o1, crit, DEV, args)
    # the reference's loop body with torch's clip and AdamW
    m2 = _latent_model().set_precision("fp32")
    o2 = torch.optim.AdamW(m2.parameters(), lr=1e-3, weight_decay=0.05)
    np.random.seed(3)
    torch.manual_seed(3)
    m2.train()
    tot, preds, labs, norms = 0.0, [], [], []
    for x, y in loader:
        x, y = x.to(DEV), y.to(DEV)
        lam = np.random.beta(1.0, 1.0)
        idx = torch.randperm(x.size(0)).to(DEV)
        xm = lam * x + (1 - lam) * x[idx]
        o2.zero_grad()
        lg = m2(xm)
        loss = lam * crit(lg, y) + (1 - lam) * crit(lg, y[idx])
        loss.backward()
        norms.append(float(torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)))
        o2.step()
        tot += loss.item() * x.size(0)
        with torch.no_grad():
            preds.extend(m2(x).argmax(1).cpu().numpy())
            labs.extend(y.cpu().numpy())
    assert max(norms) > 1.0, norms  # the clip is active in this run
    assert abs(loss1 - tot / 96) < 1e-5 * max(1.0, abs(loss1))
    # parameters: within 2.5 lr. The key third of in_proj.bias has an exactly-zero true gradient
    # (softmax is invariant to it); its rounding-noise gradient differs in sign between the two
    # optimizer implementations after step 1 and Adam turns any nonzero noise into a +-lr step.
    # Strict (1e-6) equality on identical gradients: test_fused_clip_adamw_equals_torch.
    for (k1, p1), (k2, p2) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert k1 == k2
        if p1.is_floating_point():
            torch.testing.assert_close(p1, p2, rtol=0, atol=2.5e-3, msg=k1)
    from sklearn.metrics import accuracy_score

    assert abs(acc1 - accuracy_score(labs, preds)) <= 2 / 96
    r = evaluate(m1, loader, crit, DEV)
    assert set(r) == {"loss", "accuracy", "f1_macro", "f1_weighted", "predictions", "labels"}
    assert len(r["predictions"]) == 96


def _set_grads(model, g):
    flat = model.fer_flat()
    for p in model.parameters():
        flat.attach(p)
    with torch.no_grad():
        for p in model.parameters():
            p.grad.copy_(g[id(p)])


@pytest.mark.parametrize("max_norm", [1.0, 0.05])
def test_fused_clip_adamw_equals_torch(max_norm):
    """fervit clip_grad_norm_ + FusedAdamW == torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW
    over several steps whose gradient norms lie above and below max_norm (Adam's first step is
    invariant to a global gradient scale, so a single step cannot tell clipped from unclipped)."""
    from fervit.optim import FusedAdamW, clip_grad_norm_

    m1 = _latent_model(5)
    m2 = _latent_model(5)
    m2.load_state_dict(m1.state_dict())
    m3 = _latent_model(5)  # unclipped control
    m3.load_state_dict(m1.state_dict())
    o1 = FusedAdamW(m1.parameters(), lr=1e-3, weight_decay=0.05, model=m1)
    o2 = torch.optim.AdamW(m2.parameters(), lr=1e-3, weight_decay=0.05)
    o3 = FusedAdamW(m3.parameters(), lr=1e-3, weight_decay=0.05, model=m3)
    gen = torch.Generator(device=DEV).manual_seed(11)
    for scale in (30.0, 0.001, 4.0, 200.0):
        gs = [torch.randn(p.shape, device=DEV, generator=gen) * scale for p in m1.parameters()]
        for m, o in ((m1, o1), (m2, o2), (m3, o3)):
            _set_grads(m, {id(p): g for p, g in zip(m.parameters(), gs)})
        n1 = clip_grad_norm_(m1, max_norm, optimizer=o1)
        n2 = torch.nn.utils.clip_grad_norm_(m2.parameters(), max_norm)
        torch.testing.assert_close(n1, n2, rtol=1e-5, atol=0)
        o1.step()
        o2.step()
        o3.step()
    diff_ctrl = 0.0
    for (k, p1), p2, p3 in zip(m1.state_dict().items(), m2.state_dict().values(), m3.state_dict().values()):
        if p1.is_floating_point():
            torch.testing.assert_close(p1, p2, rtol=0, atol=1e-6, msg=k)
            diff_ctrl = max(diff_ctrl, (p1 - p3).abs().max().item())
    assert diff_ctrl > 1e-4  # clipping changed the trajectory


def test_clip_coef_left_on_model_is_consumed():
    """clip_grad_norm_(model, ...) without optimizer= : a FusedAdamW bound to the model picks
    the coefficient up from the model (the trainers' call form), once."""
    from fervit.optim import FusedAdamW, clip_grad_norm_

    m = _latent_model(6)
    o = FusedAdamW(m.parameters(), lr=1e-3, model=m)
    _set_grads(m, {id(p): torch.ones_like(p) * 10 for p in m.parameters()})
    clip_grad_norm_(m, 1.0)
    assert m._fer_clip_coef is not None
    o.step()
    assert m._fer_clip_coef is None and o.clip_coef is None


def test_image_epochs_reduce_loss():
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from models_fer_vit.image_vit import ImageViT
    from train.train_image_vit import evaluate, train_epoch

    torch.manual_seed(0)
    m = ImageViT(img_size=48, embed_dim=96, depth=2, heads=4, mlp_dim=192, dropout=0.0).to(DEV)
    loader = _loader(64, (3, 48, 48), 2, 32)
    opt = FusedAdamW(m.parameters(), lr=2e-3, weight_decay=0.0, model=m)
    crit = CrossEntropyLoss(label_smoothing=0.1)
    first = evaluate(m, loader, crit, DEV)["loss"]
    for _ in range(15):
        train_epoch(m, loader, opt, crit, DEV, grad_clip=1.0)
    assert evaluate(m, loader, crit, DEV)["loss"] < first - 0.3


def test_layerwise_param_groups_cover_trainables():
    from models_fer_vit.hybrid_latent_vit import HybridLatentViT
    from train.train_hybrid_latent_vit import get_optimizer_groups

    try:
        m = HybridLatentViT(pretrained_model_name="vit_tiny_patch16_224", use_pretrained=False,
                            freeze_transformer=True, adapter_dim=16).to(DEV)
    except Exception as e:  # pragma: no cover
        pytest.skip(f"hybrid model not constructible: {e}")
    groups = get_optimizer_groups(m, 1e-4, 0.05)
    ids = {id(p) for g in groups for p in g["params"]}
    assert all(id(p) in ids for p in m.parameters() if p.requires_grad)
    assert [g["lr"] for g in groups][-1] == 5e-4 and groups[-1]["weight_decay"] == 0


def _image_model(seed=0, dropout=0.1):
    from models_fer_vit.image_vit import ImageViT

    torch.manual_seed(seed)
    m = ImageViT(img_size=48, patch_size=16, embed_dim=96, depth=2, heads=4, mlp_dim=192, dropout=dropout)
    return m.to(DEV).set_precision("bf16")


def test_reference_train_loop_bf16_with_torch_optimizer():
    """The drop-in claim on the bf16 path: `train/train_image_vit.py`'s own loop
    (train_epoch `:110-143`, torch.optim.AdamW(model.parameters()) `:270-276`, CosineAnnealingLR
    stepped per epoch `:415-417`, torch.nn.utils.clip_grad_norm_, torch.use_deterministic_algorithms
    (True) `:40`) runs unchanged on ImageViT. After every torch optimizer step the forward must read
    the updated weights (the bf16 shadow follows the parameters' version counters): the model's eval
    logits equal those of a fresh model built from its state_dict, bit for bit. The same loop with
    FusedAdamW gives the same losses and parameters within bf16 tolerance."""
    import fervit
    from models_fer_vit.image_vit import ImageViT

    loader = _loader(48, (3, 48, 48), 4, 16)
    xe = torch.randn(8, 3, 48, 48, generator=torch.Generator().manual_seed(9)).to(DEV)
    results = {}
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        for kind in ("torch", "fused"):
            fervit.manual_seed(77)  # same dropout masks in both runs
            m = _image_model(1)
            crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)
            if kind == "torch":
                opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999))
            else:
                from fervit.optim import FusedAdamW

                opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), model=m)
            sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=3)
            losses = []
            for epoch in range(3):
                m.train()
                for images, labels in loader:
                    images, labels = images.to(DEV), labels.to(DEV)
                    opt.zero_grad()
                    logits = m(images)
                    loss = crit(logits, labels)
                    loss.backward()
                    torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
                    opt.step()
                    losses.append(loss.item())
                    if kind == "torch":
                        # the forward reads the weights torch just wrote
                        m.eval()
                        with torch.no_grad():
                            got = m(xe)
                            twin = ImageViT(img_size=48, patch_size=16, embed_dim=96, depth=2, heads=4, mlp_dim=192,
                                            dropout=0.1).to(DEV).set_precision("bf16")
                            twin.load_state_dict(m.state_dict())
                            twin.eval()
                            assert torch.equal(got, twin(xe))
                        m.train()
                sched.step()
            results[kind] = (losses, {k: v.detach().clone() for k, v in m.state_dict().items()})
    finally:
        torch.use_deterministic_algorithms(prev)
    (l1, p1), (l2, p2) = results["torch"], results["fused"]
    assert l1[-1] < l1[0]
    for a, b in zip(l1, l2):
        assert abs(a - b) < 2e-2 * max(1.0, abs(a))
    for k in p1:
        if not p1[k].is_floating_point():
            continue
        a, b = p1[k], p2[k]
        if k.endswith("in_proj_bias"):
            # the key third has an exactly-zero true gradient (softmax is invariant to it): its
            # rounding noise differs between the two optimizers and Adam turns it into +-lr steps
            D = a.numel() // 3
            assert (a[D:2 * D] - b[D:2 * D]).abs().max().item() <= 2 * len(l1) * 1e-3 + 1e-6, k
            a, b = torch.cat([a[:D], a[2 * D:]]), torch.cat([b[:D], b[2 * D:]])
        torch.testing.assert_close(a, b, rtol=0, atol=3e-3, msg=k)


def test_clip_ignores_stale_grad_slots():
    """fervit clip_grad_norm_ sums the flat gradient buffer: a parameter that got a gradient in
    step 1 and none in step 2 (a stage frozen mid-run, then zero_grad(set_to_none=True)) must not
    contribute its step-1 values -- the norm equals torch.nn.utils.clip_grad_norm_'s, which skips
    `p.grad is None` (`train/train_latent_vit_v2.py:133`). Foreign `.grad` tensors count as torch
    counts them."""
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW, clip_grad_norm_

    m = _image_model(2, dropout=0.0)
    crit = CrossEntropyLoss(label_smoothing=0.1)
    o = FusedAdamW(m.parameters(), lr=1e-3, model=m)
    g = torch.Generator().manual_seed(3)
    x, y = torch.randn(8, 3, 48, 48, generator=g).to(DEV), torch.randint(0, 7, (8,), generator=g).to(DEV)
    o.zero_grad()
    crit(m(x), y).backward()
    n_all = clip_grad_norm_(m, 1e9, optimizer=o)
    torch.testing.assert_close(n_all, torch.nn.utils.clip_grad_norm_(m.parameters(), 1e9), rtol=1e-5, atol=0)
    o.step()
    # step 2: the patch embedding and the first layer are frozen (no gradient), the head gets a
    # foreign gradient tensor assigned by user code
    frozen = list(m.patch_embed.parameters()) + list(m.transformer.layers[0].parameters())
    for p in frozen:
        p.requires_grad_(False)
    o.zero_grad(set_to_none=True)
    crit(m(x), y).backward()
    assert all(p.grad is None for p in frozen)
    m.head.weight.grad = torch.full_like(m.head.weight, 0.25)
    ours = clip_grad_norm_(m, 1e9, optimizer=o)
    ref = torch.nn.utils.clip_grad_norm_(m.parameters(), 1e9)
    torch.testing.assert_close(ours, ref, rtol=1e-5, atol=0)


def test_zero_grad_drops_a_pending_clip_coefficient():
    """A clip coefficient computed for a step that is then skipped must not scale the next step's
    gradients: FusedAdamW.zero_grad clears it."""
    from fervit.optim import FusedAdamW, clip_grad_norm_

    m = _latent_model(6)
    o = FusedAdamW(m.parameters(), lr=1e-3, model=m)
    _set_grads(m, {id(p): torch.ones_like(p) * 10 for p in m.parameters()})
    clip_grad_norm_(m, 1.0)
    assert m._fer_clip_coef is not None
    o.zero_grad()  # the step is skipped
    assert m._fer_clip_coef is None and o.clip_coef is None


@pytest.mark.parametrize("prec", ["bf16", "fp32"])
def test_step_in_backward_equals_step(prec):
    """FusedAdamW.step_in_backward (each layer's update issued from the backward's gradient-ready hook on
    the weight-gradient stream) == the same optimizer's plain step() after the backward: parameters,
    AdamW moments, the bf16 shadow and its transposed copies bit for bit over three dropout train steps
    of an ImageViT (every parameter kind: patch embedding, CLS / pos, encoder layers, head)."""
    import fervit
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from models_fer_vit.image_vit import ImageViT

    g = torch.Generator().manual_seed(5)
    x = torch.randn(16, 3, 48, 48, generator=g).to(DEV)
    y = torch.randint(0, 7, (16,), generator=g).to(DEV)
    crit = CrossEntropyLoss(label_smoothing=0.1)
    out = []
    for inbw in (False, True):
        torch.manual_seed(0)
        m = ImageViT(img_size=48, patch_size=16, embed_dim=384, depth=2, heads=8, mlp_dim=1536, dropout=0.1)
        m = m.to(DEV).set_precision(prec)
        opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.05, model=m).step_in_backward(inbw)
        fervit.manual_seed(11)
        for _ in range(3):
            opt.zero_grad()
            crit(m(x), y).backward()
            opt.step()
        torch.cuda.synchronize()
        flat = m.fer_flat()
        # (the transposed copies exist only for the 2-D parameters: compare those regions)
        ht = None if flat.half_t is None else [flat.half_t_view(p).clone() for p in m.parameters() if p.dim() == 2]
        out.append((flat.data.clone(), opt._m.clone(), opt._v.clone(),
                    None if flat.half is None else flat.half.clone(), ht,
                    [opt.state[p]["step"] for p in m.parameters()]))
        opt.step_in_backward(False)
    a, b = out
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    if a[3] is not None:
        assert torch.equal(a[3].view(torch.int16), b[3].view(torch.int16))
    if a[4] is not None:
        assert all(torch.equal(u.view(torch.int16), v.view(torch.int16)) for u, v in zip(a[4], b[4]))
    assert a[5] == b[5]


@pytest.mark.parametrize("pattern", [(True, False, True, True, False, True), (False, True, False, False, True, True)])
def test_step_in_backward_switched_mid_run(pattern):
    """step_in_backward switched on and off between steps (as tools/step_ab.py does between variants) ==
    plain step() every step, bit for bit: the per-layer tables and step()'s resident table are reused only
    when every parameter's host step moved by exactly one since their last launch, so a table
    left stale by the other path is rebuilt instead of advanced with the wrong bias-correction step."""
    import fervit
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from models_fer_vit.image_vit import ImageViT

    g = torch.Generator().manual_seed(6)
    x = torch.randn(16, 3, 48, 48, generator=g).to(DEV)
    y = torch.randint(0, 7, (16,), generator=g).to(DEV)
    crit = CrossEntropyLoss(label_smoothing=0.1)
    out = []
    for pat in ((False,) * len(pattern), pattern):
        torch.manual_seed(0)
        m = ImageViT(img_size=48, patch_size=16, embed_dim=384, depth=2, heads=8, mlp_dim=1536, dropout=0.1)
        m = m.to(DEV).set_precision("bf16")
        opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.05, model=m)
        fervit.manual_seed(12)
        for inbw in pat:
            opt.step_in_backward(inbw)
            opt.zero_grad()
            crit(m(x), y).backward()
            opt.step()
        opt.step_in_backward(False)
        torch.cuda.synchronize()
        out.append((m.fer_flat().data.clone(), opt._m.clone(), opt._v.clone(),
                    [opt.state[p]["step"] for p in m.parameters()]))
    a, b = out
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert a[3] == b[3]


def test_step_in_backward_second_backward_raises():
    """Two backward passes before step() under step_in_backward (gradient accumulation) would apply only the
    first pass's gradients to the parameters the hook already updated: refused with an error."""
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from models_fer_vit.image_vit import ImageViT

    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 48, 48, generator=g).to(DEV)
    y = torch.randint(0, 7, (8,), generator=g).to(DEV)
    crit = CrossEntropyLoss()
    m = ImageViT(img_size=48, patch_size=16, embed_dim=384, depth=1, heads=8, mlp_dim=1536, dropout=0.0)
    m = m.to(DEV).set_precision("bf16")
    opt = FusedAdamW(m.parameters(), lr=1e-3, model=m).step_in_backward(True)
    try:
        opt.zero_grad()
        crit(m(x), y).backward()
        with pytest.raises(RuntimeError, match="second backward"):
            crit(m(x), y).backward()
    finally:
        from fervit import runtime
        from fervit.optim import _close_reduce_window

        opt.step_in_backward(False)
        # the raising backward dropped its queued engine callbacks: join the weight-gradient stream and
        # close the deferred-reduction window by hand so later tests start clean
        runtime.WGRAD.join_queued = False
        runtime.WGRAD.sync()
        _close_reduce_window()
        torch.cuda.synchronize()
