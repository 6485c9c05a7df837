"""Graph-replayed training steps (fervit.graph.StepGraph) against the same steps run eagerly.

* dropout 0: the replayed steps are the eager steps exactly (same kernels, same order, the
  AdamW bias-correction step taken from the device counter) -> identical losses and parameters.
* dropout > 0 with lr 0: consecutive replays of the same batch draw fresh dropout masks
  (the device step counter is mixed into every captured seed) -> the losses differ, and
  disabling dropout makes them identical again.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def make(dropout, seed=3):
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW
    from models_fer_vit.latent_vit import LatentViT

    torch.manual_seed(seed)
    m = LatentViT(embed_dim=128, depth=2, heads=2, mlp_dim=256, dropout=dropout).cuda()
    m.set_precision("bf16")
    return m, CrossEntropyLoss(label_smoothing=0.1)


def batch(B=32):
    g = torch.Generator(device="cuda").manual_seed(11)
    return torch.randn(B, 18, 512, device="cuda", generator=g), torch.randint(0, 7, (B,), device="cuda", generator=g)


def test_graph_replay_equals_eager_steps():
    from fervit.graph import StepGraph
    from fervit.optim import FusedAdamW

    x, y = batch()
    ma, crit = make(0.0)
    oa = FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.05, model=ma)
    mb, _ = make(0.0)
    ob = FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.05, model=mb)

    def step(m, o):
        o.zero_grad(set_to_none=True)
        loss = crit(m(x), y)
        loss.backward()
        o.step()
        return loss

    eager = [step(ma, oa).item() for _ in range(6)]
    sg = StepGraph(lambda: step(mb, ob), ob, warmup=2).capture()
    try:
        graphed = [step_loss.item() for step_loss in (sg.replay().clone() for _ in range(4))]
    finally:
        sg.release()
    # warm-up steps (2, eager) + 4 replays == 6 eager steps
    assert graphed == pytest.approx(eager[2:], rel=0, abs=1e-6)
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        assert (pa.detach() - pb.detach()).abs().max().item() <= 1e-6


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_graph_replays_draw_fresh_dropout_masks(p):
    from fervit.graph import StepGraph
    from fervit.optim import FusedAdamW

    x, y = batch()
    m, crit = make(p)
    o = FusedAdamW(m.parameters(), lr=0.0, weight_decay=0.0, model=m)

    def step():
        o.zero_grad(set_to_none=True)
        loss = crit(m(x), y)
        loss.backward()
        o.step()
        return loss

    sg = StepGraph(step, o, warmup=1).capture()
    try:
        losses = [sg.replay().item() for _ in range(3)]
    finally:
        sg.release()
    if p == 0.0:
        assert losses[0] == losses[1] == losses[2]
    else:
        assert len(set(losses)) == 3


def test_release_folds_replays_into_step_count():
    """After StepGraph.release the optimizer's host step counts include the replays: a
    checkpoint taken then, and eager steps after it, continue the bias correction exactly as
    an all-eager run (graph-mode step count)."""
    from fervit.graph import StepGraph
    from fervit.optim import FusedAdamW

    x, y = batch()
    ma, crit = make(0.0)
    oa = FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.05, model=ma)
    mb, _ = make(0.0)
    ob = FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.05, model=mb)

    def step(m, o):
        o.zero_grad(set_to_none=True)
        loss = crit(m(x), y)
        loss.backward()
        o.step()
        return loss

    for _ in range(8):
        step(ma, oa)
    sg = StepGraph(lambda: step(mb, ob), ob, warmup=2).capture()
    for _ in range(4):
        sg.replay()
    sg.release()
    steps = {int(v["step"]) for v in ob.state_dict()["state"].values()}
    assert steps == {6}, steps
    for _ in range(2):
        step(mb, ob)
    torch.cuda.synchronize()
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        assert (pa.detach() - pb.detach()).abs().max().item() <= 1e-6
    assert {int(v["step"]) for v in ob.state_dict()["state"].values()} == {8}


def test_graph_replay_follows_lr_scheduler():
    """An LR scheduler stepped between replays (`train/train_latent_vit_v2.py:368-370`: one
    scheduler.step() per epoch) changes the lr the captured AdamW node uses: the segment table is
    rewritten before the next replay (FusedAdamW.sync_graph_hparams), so graph and eager runs with
    the same schedule stay equal -- and differ from a run whose lr never changes."""
    from fervit.graph import StepGraph
    from fervit.optim import FusedAdamW

    x, y = batch()
    runs = []
    for mode in ("eager", "graph", "graph-const-lr"):
        m, crit = make(0.0)
        o = FusedAdamW(m.parameters(), lr=2e-3, weight_decay=0.05, model=m)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(o, T_max=4)

        def step():
            o.zero_grad(set_to_none=True)
            loss = crit(m(x), y)
            loss.backward()
            o.step()
            return loss

        if mode == "eager":
            for _ in range(2):  # the graph runs' warm-up steps
                step()
        else:
            sg = StepGraph(step, o, warmup=2).capture()
        for epoch in range(4):
            for _ in range(2):
                step() if mode == "eager" else sg.replay()
            if mode != "graph-const-lr":
                sched.step()
        if mode != "eager":
            sg.release()
        torch.cuda.synchronize()
        runs.append([p.detach().clone() for p in m.parameters()])
        if mode != "graph-const-lr":
            assert o.param_groups[0]["lr"] < 1e-4  # the schedule ran (cosine to ~0 at T_max)
    eager, graph, const = runs
    for pa, pb in zip(eager, graph):
        assert (pa - pb).abs().max().item() <= 1e-6
    assert max((pa - pc).abs().max().item() for pa, pc in zip(eager, const)) > 1e-4
