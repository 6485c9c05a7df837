"""Deferred gradient reductions (fervit.layers._ReduceDefer, csrc/misc.hip fer_reduce_defer): the
bias / LayerNorm / attention-bias gradients of a backward with the queued, batched fixed-order sums
are bit-identical to the immediate per-kernel reductions (same per-column arithmetic), for every
model family, both precisions, with dropout on (train mode) where the family has it."""
import pytest
import torch

from cases import CASES, case_inputs

pytestmark = pytest.mark.gpu


def _grads(m, x, y, defer):
    from fervit import runtime
    from fervit.layers import REDUCE

    REDUCE.enabled = defer
    try:
        m.zero_grad(set_to_none=True)
        runtime.manual_seed(1234)
        w0 = REDUCE.windows
        loss = torch.nn.functional.cross_entropy(m(x), y, label_smoothing=0.1)
        loss.backward()
        torch.cuda.synchronize()
        assert (REDUCE.windows > w0) == defer
        return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    finally:
        REDUCE.enabled = True


def _compare(m, x, y):
    a = _grads(m, x, y, True)
    b = _grads(m, x, y, False)
    assert a.keys() == b.keys() and a
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_deferred_reductions_bit_identical(name, prec):
    from test_gpu_models import build

    m, _ = build(name)
    m.set_precision(prec).train()
    x, y = case_inputs(name)
    _compare(m, x.cuda(), y.cuda())


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_deferred_reductions_hybrid(prec):
    from test_gpu_hybrid import B, L, LAT, _hybrid

    m = _hybrid().cuda()
    m.set_precision(prec).eval()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, L, LAT, generator=g).cuda()
    y = torch.randint(0, 7, (B,), generator=g).cuda()
    _compare(m, x, y)


def test_deferred_reductions_grad_accumulation():
    """Two backward passes into the same .grad (accumulate): queued sums keep stream order."""
    from test_gpu_models import build
    from fervit import runtime
    from fervit.layers import REDUCE

    name = next(iter(CASES))
    m, _ = build(name)
    m.set_precision("bf16").train()
    x, y = case_inputs(name)
    x, y = x.cuda(), y.cuda()
    out = []
    for defer in (True, False):
        REDUCE.enabled = defer
        try:
            m.zero_grad(set_to_none=True)
            runtime.manual_seed(7)
            for _ in range(2):
                torch.nn.functional.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            out.append({k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None})
        finally:
            REDUCE.enabled = True
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_reduce_defer_c_api_contract():
    """fer_reduce_defer / fer_reduce_flush driven directly: a queued sum leaves its outputs untouched
    until the flush; a second update of a queued output runs the queue first (stream order, so an
    accumulate lands on the finished value); a paused window and a partial set above the arena run
    immediately; closing the window flushes."""
    from fervit import ops
    from fervit._lib import check, lib

    M, D = 4864, 512  # LayerNorm partials 304 x 3D fp32 = 1.9 MB: a deferrable set
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.rand(D, device="cuda", generator=g) + 0.5
    b = torch.zeros(D, device="cuda")
    mean = torch.empty(M, device="cuda")
    rstd = torch.empty(M, device="cuda")
    ops.layernorm_fwd(x, w, b, 1e-5, mean=mean, rstd=rstd)

    def run(dg, db, acc=False):
        ops.layernorm_bwd(dy, x, mean, rstd, w, dgamma=dg, dbeta=db, accumulate=acc)

    g_ref, b_ref = torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    run(g_ref, b_ref)
    arena = torch.empty(16 << 18, device="cuda")  # 16 MB
    st = ops.stream()
    dg, db = torch.full((D,), 7.0, device="cuda"), torch.full((D,), 7.0, device="cuda")
    check(lib().fer_reduce_defer(1, arena.data_ptr(), arena.numel() * 4, st), "defer")
    try:
        run(dg, db)
        torch.cuda.synchronize()
        assert (dg == 7.0).all() and (db == 7.0).all()  # queued
        run(dg, db, acc=True)  # same outputs: the queue runs first, then this one
        torch.cuda.synchronize()
        assert torch.equal(dg, g_ref + g_ref) and torch.equal(db, b_ref + b_ref)
        check(lib().fer_reduce_defer(2, None, 0, None), "pause")
        dg2, db2 = torch.full((D,), 7.0, device="cuda"), torch.full((D,), 7.0, device="cuda")
        run(dg2, db2)  # paused: immediate
        torch.cuda.synchronize()
        assert torch.equal(dg2, g_ref) and torch.equal(db2, b_ref)
        check(lib().fer_reduce_defer(1, arena.data_ptr(), arena.numel() * 4, st), "resume")
        dg3, db3 = torch.full((D,), 7.0, device="cuda"), torch.full((D,), 7.0, device="cuda")
        run(dg3, db3)
        check(lib().fer_reduce_flush(), "flush")
        torch.cuda.synchronize()
        assert torch.equal(dg3, g_ref) and torch.equal(db3, b_ref)
        run(dg3, db3, acc=True)  # queued again; closing the window flushes it
    finally:
        check(lib().fer_reduce_defer(0, None, 0, None), "close")
    torch.cuda.synchronize()
    assert torch.equal(dg3, g_ref + g_ref)
    small = torch.empty(65536 // 4, device="cuda")  # a 64 KB arena: the 1.9 MB set cannot be taken
    dg4, db4 = torch.full((D,), 7.0, device="cuda"), torch.full((D,), 7.0, device="cuda")
    check(lib().fer_reduce_defer(1, small.data_ptr(), small.numel() * 4, st), "defer")
    try:
        run(dg4, db4)
        torch.cuda.synchronize()
        assert torch.equal(dg4, g_ref) and torch.equal(db4, b_ref)
    finally:
        check(lib().fer_reduce_defer(0, None, 0, None), "close")


def test_deferred_window_after_backward_exception():
    """A backward that raises drops its queued end-of-backward callback: the window it
    opened must not swallow the next backward's sums. The next backward's gradients equal the
    immediate path's, and an optimizer step / clip after the failed backward closes the window."""
    from fervit.layers import REDUCE
    from fervit.optim import clip_grad_norm_
    from test_gpu_models import build

    m, _ = build("latent_vit")
    m.set_precision("bf16").train()
    x, y = case_inputs("latent_vit")
    x, y = x.cuda(), y.cuda()
    ref = _grads(m, x, y, False)

    def boom(_g):
        raise RuntimeError("injected backward failure")

    for after in ("backward", "clip"):
        m.zero_grad(set_to_none=True)
        xr = x.clone().requires_grad_(True)
        xr.register_hook(boom)  # fires after every layer backward opened the window
        loss = torch.nn.functional.cross_entropy(m(xr), y, label_smoothing=0.1)
        with pytest.raises(RuntimeError, match="injected"):
            loss.backward()
        assert REDUCE.open  # its callback was dropped with the exception
        if after == "clip":
            clip_grad_norm_(m, 1.0)
            assert not REDUCE.open
        got = _grads(m, x, y, True)
        assert not REDUCE.open
        assert got.keys() == ref.keys()
        for k in ref:
            assert torch.equal(got[k], ref[k]), (after, k)
