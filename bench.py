"""Headline benchmark: training images/s of ViT-B/16 (224x224 RGB, per-GPU bs=256,
dropout 0.1, label-smoothed CE, AdamW) — BASELINE.json configs[2] — on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config vit_base_224|latent_vit|image_vit_48]
    (N>1: torch.distributed.run, one rank per GPU, RCCL all-reduce over xGMI)

A step = zero_grad -> forward -> CE -> backward (bucketed all-reduce overlapped when N>1)
-> fused AdamW, on synthetic data already resident in HBM. Rank 0 prints one JSON line.

roofline: the dominant kernel is the bf16 MFMA GEMM of the FFN up-projection
(linear1, [B*197 x 768] x [3072 x 768]^T + bias + GELU + dropout epilogue). Its launches
inside the timed region are bracketed by HIP events on the launch stream; achieved =
2*M*N*K / mean launch time vs the dense bf16 MFMA peak (MI355X_MICROARCH.md: 256 CU x 4
SIMD x 1024 FLOP/clk x 2.4 GHz = 2516.6 TFLOP/s). `step_mfma_frac` is the whole step's
algorithmic GEMM+attention FLOPs (105.38 GFLOP/img fwd+bwd) / step time / peak.
cpu_baseline: the CPU oracle (oracle/vit_oracle.py, same model, fp32, dropout 0.1, AdamW)
timed on the host cores for a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12  # 2516.6
METRIC = "training images/sec at 1/2/4/8 MI355X, ViT-B/16 bs=256; fwd+bwd step ms"

CONFIGS = {
    # name: (model kind, ctor, per-GPU batch, input shape, workload description)
    "vit_base_224": ("image", dict(img_size=224, patch_size=16, embed_dim=768, depth=12, heads=12, mlp_dim=3072,
                                   dropout=0.1), 256, (3, 224, 224),
                     "image_vit ViT-B/16, 224x224 RGB AffectNet-shaped synthetic, bs=256/GPU, train step "
                     "(fwd+bwd+AdamW), dropout 0.1, CE label_smoothing 0.1"),
    "latent_vit": ("latent", dict(), 256, (18, 512),
                   "latent_vit d6/h8 e512 on synthetic w+ latents (18x512), bs=256/GPU, train step"),
    "image_vit_48": ("image", dict(img_size=48, patch_size=16, embed_dim=384, depth=6, heads=8, mlp_dim=1536,
                                   dropout=0.1), 64, (3, 48, 48),
                     "image_vit d6/h8 e384, 48x48 FER-2013-shaped synthetic, bs=64, train step"),
    "hybrid_latent_vit": ("hybrid", dict(), 256, (18, 512),
                          "hybrid_latent_vit timm-B/16 blocks frozen + adapter 64, w+ latents, bs=256/GPU, "
                          "train step (CE, AdamW on the trainable parameters)"),
    "expression_aware_vit": ("expr", dict(), 256, (18, 512),
                             "expression_aware_vit: decomposer (7 seeded unit directions, all_classes, "
                             "expr_only) + SPE + LEAM + hybrid timm-B/16 frozen + adapter 64, bs=256/GPU"),
}


def gemm_flops_per_img(D, L, F, N, patch_k=None, n_patch=None):
    per_layer = 2 * N * D * 3 * D + 4 * N * N * D + 2 * N * D * D + 4 * N * D * F
    f = L * per_layer + (2 * n_patch * patch_k * D if patch_k else 0)
    return 3 * f  # fwd + bwd (dgrad + wgrad)


def build(cfg_name, device):
    from fervit.loss import CrossEntropyLoss
    from fervit.optim import FusedAdamW

    kind, ctor, B, shape, desc = CONFIGS[cfg_name]
    ls = 0.1
    if kind == "image":
        from models_fer_vit.image_vit import ImageViT

        m = ImageViT(num_classes=7, **ctor)
    elif kind == "latent":
        from models_fer_vit.latent_vit import LatentViT

        m = LatentViT(**ctor)
    else:  # SURVEY §8(d) cfg4 / cfg5 (the hybrid trainers use no label smoothing)
        from models_fer_vit.hybrid_latent_vit import create_hybrid_latent_vit

        ls = 0.0
        vit = create_hybrid_latent_vit(model_size="base", use_pretrained=False, freeze_transformer=True,
                                       use_adapter=True, adapter_dim=64)
        if kind == "hybrid":
            m = vit
        else:
            from models_fer_vit.expression_aware_vit import ExpressionAwareViT
            from models_fer_vit.latent_decomposer import LatentDecomposer

            g = torch.Generator().manual_seed(7)
            dirs = {c: torch.nn.functional.normalize(torch.randn(18, 512, generator=g).view(-1), dim=0).view(18, 512)
                    for c in range(7)}
            m = ExpressionAwareViT(LatentDecomposer(dirs), vit, output_mode="expr_only",
                                   decompose_mode="all_classes", use_spe=True, use_leam=True)
    m = m.to(device)
    m.set_precision("bf16")
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.05, model=m)
    return m, opt, CrossEntropyLoss(label_smoothing=ls), B, shape, desc


class GemmProbe:
    """HIP events around the launches of one GEMM signature, on the launch stream."""

    def __init__(self, M, N, K):
        self.sig = (M, N, K)
        self.events = []
        self.on = False

    def __call__(self, desc, launch):
        if not self.on or (desc.M, desc.N, desc.K) != self.sig or not (desc.a_kc and desc.b_kc):
            return launch()
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        r = launch()
        b.record(s)
        self.events.append((a, b))
        return r

    def mean_ms(self):
        ts = [a.elapsed_time(b) for a, b in self.events]
        return sum(ts) / max(1, len(ts)), len(ts)


def pmc_traffic(timeout_s=120):
    """HBM bytes per launch of the roofline kernel from rocprofv3 PMC counters, one counter per
    pass (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE in KiB; on gfx950 FETCH_SIZE reads half the
    bytes of a 16 B/lane streaming read -- the GEMM's LDS-DMA operand loads -- so it is doubled;
    WRITE_SIZE is exact for 16 B/lane stores). Runs tools/traffic_probe.py as a CHILD process under
    rocprofv3 before this process touches the GPU. Returns (bytes, detail) or (None, reason)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    probe = os.path.join(ROOT, "tools", "traffic_probe.py")
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"pmc_{ctr}_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", ctr, "--output-format", "csv", "-d", d,
               "-o", "p", "--", sys.executable, probe]
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout_s + 30)
        except Exception as ex:  # noqa: BLE001
            return None, f"{ctr} pass failed: {ex}"
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            return None, f"{ctr} pass rc={r.returncode}: {r.stdout.decode(errors='replace')[-300:]}"
        per = []
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if "gemm" in row.get("Kernel_Name", "") and row.get("Counter_Name", "") == ctr:
                    per.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not per:
            return None, f"{ctr}: no gemm dispatch in the counter CSV"
        per.sort()
        vals[ctr] = per[len(per) // 2]  # median over the probe's launches (KiB)
    read_b = 2.0 * vals["FETCH_SIZE"] * 1024
    write_b = vals["WRITE_SIZE"] * 1024
    return read_b + write_b, {"read_bytes": read_b, "write_bytes": write_b, "fetch_size_kib": vals["FETCH_SIZE"],
                              "write_size_kib": vals["WRITE_SIZE"], "method": "rocprofv3 --pmc, one counter per "
                              "pass, median over 6 launches; read = 2*FETCH_SIZE (gfx950 16 B/lane correction)"}


def cpu_baseline(cfg_name, budget_s=20.0):
    """Oracle train step (fp32, torch CPU ops) on a bounded sample of the workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vit_oracle as O

    kind, ctor, B, shape, desc = CONFIGS[cfg_name]
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(42)
    if kind != "image":
        return None
    D, L, H, F, P = ctor["embed_dim"], ctor["depth"], ctor["heads"], ctor["mlp_dim"], ctor["patch_size"]
    C = shape[0]
    n = (shape[1] // P) ** 2
    p = {"patch_embed.proj.weight": torch.randn(D, C, P, P, generator=g) * 0.02,
         "patch_embed.proj.bias": torch.zeros(D), "cls_token": torch.randn(1, 1, D, generator=g) * 0.02,
         "pos_embed": torch.randn(1, n + 1, D, generator=g) * 0.02, "norm.weight": torch.ones(D),
         "norm.bias": torch.zeros(D), "head.weight": torch.randn(7, D, generator=g) * 0.02, "head.bias": torch.zeros(7)}
    for i in range(L):
        pre = f"transformer.layers.{i}."
        for k, s in (("self_attn.in_proj_weight", (3 * D, D)), ("self_attn.out_proj.weight", (D, D)),
                     ("linear1.weight", (F, D)), ("linear2.weight", (D, F))):
            p[pre + k] = torch.randn(*s, generator=g) * 0.02
        for k, s in (("self_attn.in_proj_bias", 3 * D), ("self_attn.out_proj.bias", D), ("linear1.bias", F),
                     ("linear2.bias", D), ("norm1.bias", D), ("norm2.bias", D)):
            p[pre + k] = torch.zeros(s)
        p[pre + "norm1.weight"] = torch.ones(D)
        p[pre + "norm2.weight"] = torch.ones(D)
    for t in p.values():
        t.requires_grad_(True)
    m = {k: torch.zeros_like(v) for k, v in p.items()}
    v2 = {k: torch.zeros_like(v) for k, v in p.items()}
    bs = 2 if D >= 768 else 16
    x = torch.randn(bs, *shape, generator=g)
    y = torch.randint(0, 7, (bs,), generator=g)
    step = [0]

    def one():
        for t in p.values():
            t.grad = None
        logits = O.image_vit_forward(x, p, P, H, L, p_drop=0.1)
        O.cross_entropy(logits, y, 0.1).backward()
        step[0] += 1
        with torch.no_grad():
            for k, t in p.items():
                O.adamw_step(t, t.grad, m[k], v2[k], step[0], 1e-3, wd=0.05)

    one()  # warm-up
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 2:
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
        if len(times) >= 20:
            break
    times.sort()
    med = times[len(times) // 2]
    return {"value": bs / med, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle ViT train step (fwd+bwd+AdamW, fp32, dropout 0.1) at bs={bs}, "
                      f"{len(times)} timed steps, median {med * 1e3:.0f} ms/step, torch {torch.__version__}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="vit_base_224", choices=list(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the whole step as a HIP graph (auto: on for the launch-bound small configs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    traffic, traffic_detail = None, "not measured (N>1 or --no-traffic)"
    if world == 1 and not args.no_traffic and args.config == "vit_base_224":
        # child rocprofv3 passes first: this process has not initialised the GPU yet
        traffic, traffic_detail = pmc_traffic()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    import fervit
    from fervit import ops

    fervit.manual_seed(1234 + rank)
    torch.manual_seed(42)
    model, opt, crit, B, shape, desc = build(args.config, device)
    net = model
    if world > 1:
        from fervit.ddp import DistributedDataParallel

        net = DistributedDataParallel(model)
    g = torch.Generator(device=device).manual_seed(42 + rank)
    x = torch.randn(B, *shape, device=device, generator=g)
    y = torch.randint(0, 7, (B,), device=device, generator=g)

    kind, ctor = CONFIGS[args.config][:2]
    if kind == "image":
        D, L, F = ctor["embed_dim"], ctor["depth"], ctor["mlp_dim"]
        N = (ctor["img_size"] // ctor["patch_size"]) ** 2 + 1
        flops_img = gemm_flops_per_img(D, L, F, N, 3 * ctor["patch_size"] ** 2, N - 1)
    elif kind == "latent":
        D, L, F, N = 512, 6, 2048, 19
        flops_img = gemm_flops_per_img(D, L, F, N) + 3 * 2 * 18 * 512 * 512
    else:
        # frozen trunk: fwd + dgrad only (2x its fwd); trainable input_proj, adapters, head: 3x
        D, L, F, N = 768, 12, 3072, 19
        trunk = gemm_flops_per_img(D, L, F, N) // 3
        adapters = L * 2 * N * (2 * D * 64)
        flops_img = 2 * trunk + 3 * (adapters + 2 * 18 * 512 * D + 2 * D * 7)
    probe = GemmProbe(B * N, F, D)
    ops.LAUNCH_PROBE = probe

    def step():
        opt.zero_grad()
        loss = crit(net(x), y)
        loss.backward()
        opt.step()
        return loss

    use_graph = args.graph == "on" or (args.graph == "auto" and args.config != "vit_base_224" and world == 1)
    if use_graph:
        # the roofline kernel is timed in eager warm-up steps (HIP events cannot bracket single
        # launches inside a replayed graph); the timed region replays the captured step
        from fervit.graph import StepGraph

        probe.on = True
        for _ in range(args.warmup):
            step()
        probe.on = False
        graph = StepGraph(step, opt, warmup=1).capture()
        run = graph.replay
    else:
        for _ in range(args.warmup):
            step()
        run = step
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    probe.on = not use_graph
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    probe.on = False
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    gemm_ms, nlaunch = probe.mean_ms()
    ms = el / args.steps * 1e3
    imgs = world * B * args.steps / el
    step_tflops = flops_img * B / (ms / 1e3) / 1e12
    gemm_flop = 2.0 * B * N * F * D
    # bytes the fc1 launch must move at minimum: X [BN x D] + W1 [F x D] read, pre + out [BN x F] written (bf16)
    algo_bytes = 2 * (B * N * D + F * D + 2 * B * N * F)
    achieved = gemm_flop / (gemm_ms / 1e3) / 1e12
    lossv = loss.item()
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.config)
        out = {
            "metric": METRIC, "value": round(imgs, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (N(0,1) inputs, uniform labels), random init",
            "config": {"workload": desc, "per_gpu_batch": B, "global_batch": B * world, "tokens": N,
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "kernel": f"gemm_bf16 linear1 fwd [{B * N}x{D}]x[{F}x{D}]^T",
                         "achieved": round(achieved, 1), "peak": round(PEAK_BF16_TFLOPS, 1), "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_detail": traffic_detail,
                         "algorithmic_bytes": algo_bytes,
                         "launches_timed": nlaunch, "mean_launch_ms": round(gemm_ms, 4)},
            "launch": "hipGraph replay of the whole step" if use_graph else "eager (one host launch per kernel)",
            "step_mfma_frac": round(step_tflops / PEAK_BF16_TFLOPS, 4),
            "step_tflops": round(step_tflops, 1),
            "final_loss": round(lossv, 4),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
