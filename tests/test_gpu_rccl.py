"""The DDP reducer on the real backend: a 1-rank "nccl" (= RCCL) process group on the test box's
GPU (the driver's 1/2/4/8-GPU bench is the only multi-rank RCCL run; the reference itself is
single-device, `/root/reference/train/train_image_vit.py:183`). Exercises fervit/ddp.py's nccl
branch -- ReduceOp.AVG on the side stream, the bf16 wire casts, `work.wait` and the compute
stream's join -- on a bf16 ViT with FusedAdamW: after 3 steps the wrapped model must equal an
unwrapped twin bit for bit (fp32 wire: AVG over one rank is the identity; gradients equal at every
step) or, on the bf16 wire, have the first step's gradients equal to the bf16 round trip of the
twin's, and bucket all-reduces must be issued while the
backward is still running (overlap), not all at its end."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, wire, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "fer-vit_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from fervit import ddp as D
        from fervit import runtime
        from fervit.loss import CrossEntropyLoss
        from fervit.optim import FusedAdamW
        from models_fer_vit.image_vit import ImageViT

        def model():
            torch.manual_seed(0)
            m = ImageViT(img_size=48, patch_size=16, embed_dim=192, depth=3, heads=4, mlp_dim=384, dropout=0.0)
            return m.to(dev).set_precision("bf16")

        g = torch.Generator().manual_seed(5)
        xs = [torch.randn(16, 3, 48, 48, generator=g).to(dev) for _ in range(3)]
        ys = [torch.randint(0, 7, (16,), generator=g).to(dev) for _ in range(3)]
        crit = CrossEntropyLoss(label_smoothing=0.1)
        wire_dt = getattr(torch, wire)

        ref = model()
        ref_opt = FusedAdamW(ref.parameters(), lr=1e-3, weight_decay=0.05, model=ref)
        m = model()
        net = D.DistributedDataParallel(m, bucket_cap_mb=0.25, grad_dtype=wire_dt)
        opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.05, model=m)
        events = []
        orig_launch = D.Reducer._launch

        def launch(self, b):
            events.append(("launch", self.buckets.index(b)))
            return orig_launch(self, b)

        D.Reducer._launch = launch
        runtime.register_grad_ready_hook(lambda ps: events.append(("ready", len(ps))))
        grad_ok = []
        for i in range(3):
            ref_opt.zero_grad()
            crit(ref(xs[i]), ys[i]).backward()
            opt.zero_grad()
            events.clear()
            crit(net(xs[i]), ys[i]).backward()
            torch.cuda.synchronize()
            nb = len(net.reducer.buckets)
            # every bucket launched, at least one while later layers' gradients were still coming
            launched = [e for e in events if e[0] == "launch"]
            last_ready = max(k for k, e in enumerate(events) if e[0] == "ready")
            first_launch = min(k for k, e in enumerate(events) if e[0] == "launch")
            overlap = first_launch < last_ready and len(launched) == nb
            # fp32 wire: every step (the replicas stay identical); bf16 wire: the first step (after
            # it the twin that saw exact gradients has moved to different parameters)
            if wire == "float32" or i == 0:
                for p, r in zip(m.parameters(), ref.parameters()):
                    want = r.grad if wire == "float32" else r.grad.to(torch.bfloat16).float()
                    grad_ok.append(bool(torch.equal(p.grad, want)))
            ref_opt.step()
            opt.step()
        torch.cuda.synchronize()
        same = all(torch.equal(p, r) for p, r in zip(m.parameters(), ref.parameters()))
        q.put(("ok", nb, overlap, all(grad_ok), same, dist.get_backend()))
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put(("error", traceback.format_exc()[-2000:], str(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["float32", "bfloat16"])
def test_rccl_one_rank_reducer(wire):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), wire, q))
    p.start()
    res = q.get(timeout=180)
    p.join(timeout=60)
    assert res[0] == "ok", res[1]
    _, nb, overlap, grads_equal, same, backend = res
    assert backend == "nccl"
    assert nb > 2, nb  # several buckets, so the overlap check means something
    assert overlap
    assert grads_equal
    if wire == "float32":
        assert same  # AVG over one rank is the identity: the replicas stay bit-identical


def _graph_worker(port, wire, q):
    """StepGraph over the DDP-wrapped model: the bucket all-reduces (RCCL, side stream) are captured
    into the step graph with the rest of the step; replays must equal eager DDP steps and the
    unwrapped model bit for bit (dropout 0, fp32 wire; bf16 wire: graph == eager DDP)."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "fer-vit_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from fervit import ddp as D
        from fervit.graph import StepGraph
        from fervit.loss import CrossEntropyLoss
        from fervit.optim import FusedAdamW
        from models_fer_vit.image_vit import ImageViT

        def model():
            torch.manual_seed(0)
            m = ImageViT(img_size=48, patch_size=16, embed_dim=192, depth=3, heads=4, mlp_dim=384, dropout=0.0)
            return m.to(dev).set_precision("bf16")

        g = torch.Generator().manual_seed(6)
        xs = [torch.randn(16, 3, 48, 48, generator=g).to(dev) for _ in range(4)]
        ys = [torch.randint(0, 7, (16,), generator=g).to(dev) for _ in range(4)]
        crit = CrossEntropyLoss(label_smoothing=0.1)
        wire_dt = getattr(torch, wire)

        def wrapped():
            m = model()
            return m, D.DistributedDataParallel(m, bucket_cap_mb=0.25, grad_dtype=wire_dt), \
                FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.05, model=m)

        ref = model()
        ref_opt = FusedAdamW(ref.parameters(), lr=1e-3, weight_decay=0.05, model=ref)
        me, ne, oe = wrapped()  # eager DDP
        mg, ng, og = wrapped()  # graph-replayed DDP
        sx, sy = xs[0].clone(), ys[0].clone()  # the graph's static batch

        def step(net, opt, x, y):
            opt.zero_grad()
            loss = crit(net(x), y)
            loss.backward()
            opt.step()
            return loss

        graph = StepGraph(lambda: step(ng, og, sx, sy), og, warmup=1).capture()  # one eager step on batch 0
        step(ne, oe, xs[0], ys[0])
        step(ref, ref_opt, xs[0], ys[0])
        eq_eager, eq_ref = [], []
        for i in range(1, 4):
            sx.copy_(xs[i])
            sy.copy_(ys[i])
            graph.replay()
            step(ne, oe, xs[i], ys[i])
            step(ref, ref_opt, xs[i], ys[i])
            torch.cuda.synchronize()
            eq_eager.append(all(torch.equal(a, b) for a, b in zip(mg.parameters(), me.parameters())))
            eq_ref.append(all(torch.equal(a, b) for a, b in zip(mg.parameters(), ref.parameters())))
        graph.release()
        q.put(("ok", eq_eager, eq_ref, len(ng.reducer.buckets)))
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put(("error", traceback.format_exc()[-2000:], str(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["float32", "bfloat16"])
def test_rccl_one_rank_step_graph(wire):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_graph_worker, args=(_port(), wire, q))
    p.start()
    res = q.get(timeout=180)
    p.join(timeout=60)
    assert res[0] == "ok", res[1]
    _, eq_eager, eq_ref, nb = res
    assert nb > 2, nb
    assert all(eq_eager), eq_eager  # captured all-reduces == eager DDP, every replay
    if wire == "float32":
        assert all(eq_ref), eq_ref  # == the unwrapped model (AVG over one rank is the identity)
