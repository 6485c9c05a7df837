"""Data parallelism with device tensors: two processes sharing the one GPU of the
test box, gloo process group (RCCL cannot run two ranks on one device; the reducer's device
path is the same: flat-buffer buckets all-reduced on a side HIP stream behind events, the
compute stream waiting before the optimizer). Every rank must see the gradient of the whole
batch, and FusedAdamW steps must keep the replicas identical."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from models_fer_vit.image_vit import ImageViT

    torch.manual_seed(0)
    m = ImageViT(img_size=48, embed_dim=96, depth=2, heads=4, mlp_dim=192, dropout=0.0).cuda()
    m.set_precision("fp32")
    return m


def _worker(rank, world, port, q, wire):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "fer-vit_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fervit.ddp import DistributedDataParallel
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW

    g = torch.Generator().manual_seed(123)
    x = torch.randn(8, 3, 48, 48, generator=g).cuda()
    y = torch.randint(0, 7, (8,), generator=g).cuda()
    crit = CrossEntropyLoss(label_smoothing=0.1)
    ref = _model()
    crit(ref(x), y).backward()
    ref_g = [p.grad.detach().clone() for p in ref.parameters()]
    m = _model()
    if rank == 1:  # rank 0's parameters must win the initial broadcast
        with torch.no_grad():
            for p in m.parameters():
                p.add_(0.5)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.05, grad_dtype=getattr(torch, wire))
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    crit(ddp(xs), ys).backward()
    err = max(((a.grad - b).norm() / (b.norm() + 1e-12)).item() for a, b in zip(m.parameters(), ref_g))
    opt = FusedAdamW(m.parameters(), lr=1e-3, model=m)
    opt.step()
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        crit(ddp(xs), ys).backward()
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    same = bool(torch.equal(gathered[0], gathered[1]))
    torch.cuda.synchronize()
    q.put((rank, err, same))
    dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["float32", "bfloat16"])
def test_ddp_device_gradients_and_replicas(wire):
    """bfloat16: buckets cast by the libfervit kernels on the side stream, reduced in bf16."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, wire)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, err, same in res:
        assert err < (1e-5 if wire == "float32" else 1e-2), (rank, err)
        assert same, rank
