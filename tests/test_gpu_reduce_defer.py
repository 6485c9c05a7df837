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
