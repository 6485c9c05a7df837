"""Checkpoint round trip in the reference's format (`utils/experiment_logger.py:121-145`,
legacy serialization; `eval/evaluate_model.py:117-122` key names): a run interrupted by
save -> fresh model + optimizer -> load continues exactly like the uninterrupted run, and the
optimizer state is torch.optim.AdamW-compatible (torch's AdamW resumes from it)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from models_fer_vit.latent_vit import LatentViT

    torch.manual_seed(seed)
    m = LatentViT(embed_dim=128, depth=2, heads=2, mlp_dim=256, dropout=0.0).cuda()
    o = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.05, model=m)
    return m, o, CrossEntropyLoss(label_smoothing=0.1)


def _steps(m, o, crit, x, y, n):
    for _ in range(n):
        o.zero_grad(set_to_none=True)
        crit(m(x), y).backward()
        o.step()


def test_resume_from_checkpoint_equals_uninterrupted(tmp_path):
    from fervit.checkpoint import load_checkpoint, save_checkpoint

    g = torch.Generator(device="cuda").manual_seed(1)
    x, y = torch.randn(16, 18, 512, device="cuda", generator=g), torch.randint(0, 7, (16,), device="cuda")
    ma, oa, crit = _setup()
    _steps(ma, oa, crit, x, y, 5)
    mb, ob, _ = _setup()
    _steps(mb, ob, crit, x, y, 3)
    path = str(tmp_path / "last_model.pt")
    save_checkpoint(path, mb, ob, epoch=3, metrics={"val_f1": 0.5}, config={"model": {"embed_dim": 128}},
                    run_id="runs/x")
    raw = open(path, "rb").read(2)
    assert raw != b"PK"  # legacy (non-zip) serialization, as the reference writes it
    mc, oc, _ = _setup(seed=7)  # different init: everything must come from the file
    ck = load_checkpoint(path, mc, oc)
    assert ck["epoch"] == 3 and ck["metrics"]["val_f1"] == 0.5 and ck["run_id"] == "runs/x"
    _steps(mc, oc, crit, x, y, 2)
    for pa, pc in zip(ma.parameters(), mc.parameters()):
        assert (pa.detach() - pc.detach()).abs().max().item() <= 1e-6


def test_optimizer_state_is_torch_adamw_format(tmp_path):
    from fervit.checkpoint import save_checkpoint

    g = torch.Generator(device="cuda").manual_seed(2)
    x, y = torch.randn(8, 18, 512, device="cuda", generator=g), torch.randint(0, 7, (8,), device="cuda")
    m, o, crit = _setup()
    _steps(m, o, crit, x, y, 2)
    ck = save_checkpoint(str(tmp_path / "c.pt"), m, o, epoch=1)
    sd = ck["optimizer_state_dict"]
    st = sd["state"][0]
    assert set(st) >= {"step", "exp_avg", "exp_avg_sq"} and float(st["step"]) == 2.0
    assert st["exp_avg"].shape == next(m.parameters()).shape
    ref = torch.optim.AdamW([p.detach().clone().requires_grad_(True) for p in m.parameters()], lr=1e-3,
                            weight_decay=0.05)
    ref.load_state_dict(sd)  # torch's own AdamW accepts the state
    assert torch.equal(ref.state[ref.param_groups[0]["params"][0]]["exp_avg"].cpu(), st["exp_avg"])
