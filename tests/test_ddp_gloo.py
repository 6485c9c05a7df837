"""Multi-process data parallelism on CPU (gloo, world_size 2): the fervit reducer
(bucketed all-reduce of a flat gradient buffer) must give every rank the
gradient of the concatenated global batch — the same as one process on all samples."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 32), torch.nn.GELU(),
                               torch.nn.Linear(32, 7))


def _worker(rank, world, port, q, bucket_mb, wire=torch.float32):
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fervit.ddp import DistributedDataParallel

    m = _model()
    if rank == 1:  # different init on rank 1: DDP must broadcast rank 0's parameters
        with torch.no_grad():
            for p in m.parameters():
                p.add_(1.0)
    ddp = DistributedDataParallel(m, bucket_cap_mb=bucket_mb, grad_dtype=wire)
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 16, generator=g)
    y = torch.randint(0, 7, (8,), generator=g)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    for _ in range(2):
        for p in m.parameters():
            p.grad = None
        torch.nn.functional.cross_entropy(ddp(xs), ys).backward()
    q.put((rank, [p.grad.numpy().copy() for p in m.parameters()], [p.detach().numpy().copy() for p in m.parameters()]))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb,wire", [(1e-3, torch.float32), (32.0, torch.float32), (1e-3, torch.bfloat16)])
def test_ddp_gradients_equal_single_process(bucket_mb, wire):
    """fp32 wire: equal to the single-process gradient to 1e-6. bf16 wire: every rank holds the
    same gradient (bit-identical across ranks), within bf16 rounding of the single-process one."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, bucket_mb, wire)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, w)) for r, g, w in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
    ref = _model()
    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 16, generator=g)
    y = torch.randint(0, 7, (8,), generator=g)
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    for r in range(world):
        grads, weights = res[r]
        for a, b in zip(grads, [p.grad for p in ref.parameters()]):
            if wire == torch.float32:
                assert torch.allclose(torch.from_numpy(a), b, atol=1e-6), r
            else:  # two bf16 roundings (cast, sum) of each half-batch gradient
                assert torch.allclose(torch.from_numpy(a), b, rtol=2e-2, atol=2e-3), r
        for a, b in zip(grads, res[0][0]):
            assert (a == b).all(), r
        for a, b in zip(weights, ref.parameters()):
            assert torch.equal(torch.from_numpy(a), b.detach())
