"""Headline benchmark: training images/s of ViT-B/16 (224x224 RGB, per-GPU bs=256,
dropout 0.1, label-smoothed CE, AdamW) — BASELINE.json configs[2] — on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config vit_base_224|latent_vit|image_vit_48|...]

--gpus N > 1 without a torch.distributed environment: this process starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a CHILD (it never touches
the GPU itself) and relays rank 0's JSON line; under torch.distributed.run (the driver's
launch) every rank runs the step on its own GPU, RCCL all-reduce over xGMI.

A step = zero_grad -> forward -> CE -> backward (bucketed all-reduce overlapped when N>1)
-> fused AdamW, on synthetic data already resident in HBM. W untimed warm-up steps, then K
steps bracketed by barrier + synchronize (value = all ranks' images / the max over ranks of
that time); one HIP event per step boundary gives the per-step median / p10 / p90.

roofline: the dominant kernel is `gemm_8ph_kernel`, the bf16 MFMA GEMM of every forward and
input-gradient linear (QKV, out-proj, fc1, fc2, patch embed; ~55 % of the step). Its launches
are timed in a separate PROBE phase after the timed region (HIP events on the launch stream
around each launch, so the timed region carries no probe events; weight gradients on the compute
stream during the probe, so no launch shares the chip with a concurrent one): achieved = sum over one
step's 8-phase launches of 2*M*N*K / sum of their durations, vs the dense bf16 MFMA peak
(MI355X_MICROARCH.md: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz = 2516.6 TFLOP/s).
`traffic` = HBM bytes per launch of that kernel from rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE; one counter per pass, child processes run before this process touches the GPU).
`step_mfma_frac` is the whole step's algorithmic GEMM+attention FLOPs (SURVEY §8d:
105.38 GFLOP/img fwd+bwd) / step time / peak.
cpu_baseline: the CPU oracle (oracle/vit_oracle.py, same model, fp32, dropout 0.1, AdamW)
timed on the host cores for a bounded sample (rank 0, N=1 only); cpu_baseline_cfg1 the same
for BASELINE configs[0] (48 px ImageViT d6/h8, bs=64, the reference's CPU-runnable case).
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


def is_8ph(d) -> bool:
    """The launches csrc/gemm.hip sends to gemm_8ph_kernel (automatic configuration): bf16,
    both operands K-contiguous, a grid of >= 256 256x256 tiles (or K >= 8192)."""
    t256 = -(-d.M // 256) * -(-d.N // 256)
    return d.dtype == 0 and bool(d.a_kc) and bool(d.b_kc) and (d.K >= 8192 or t256 >= 256)


def gemm_algo_bytes(d, e) -> int:
    """Minimum HBM bytes of one GEMM launch: A and B read once, every epilogue operand read once
    (bias, res, aux rows), the output (and pre-activation) written once, at storage dtypes."""
    out_b = 4 if e.c_f32 else 2
    n = 2 * (d.M * d.K + d.N * d.K) + d.M * d.N * out_b * (2 if e.accumulate else 1)
    if e.bias:
        n += 4 * d.N
    for ptr_ in (e.pre, e.res, e.aux):
        if ptr_:
            n += 2 * d.M * d.N
    return n


class GemmProbe:
    """HIP events around every gemm_8ph launch, on the launch stream (probe phase only)."""

    def __init__(self, probe_all=False):
        self.rec = []
        self.other = []  # --probe-all: every other GEMM launch too (stderr table, not the JSON line)
        self.all = probe_all
        self.on = False

    def __call__(self, d, e, launch):
        if not self.on or not (is_8ph(d) or self.all):
            return launch()
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        r = launch()
        b.record(s)
        act, gate = e.act & 15, bool(e.act & 16)
        parts = [n for n, on in (("bias", e.bias), ("gelu" if act == 1 else "relu", act), ("drop", e.drop_thresh),
                                 ("gate" if gate else "pre", e.pre), ("x gate" if e.aux_act == 3 else "act'", e.aux),
                                 ("res", e.res), ("colsum", e.colsum)) if on]
        kind = "epi:" + ("+".join(parts) or "none")
        if not is_8ph(d):
            lay = ("K" if d.a_kc else "M") + ("K" if d.b_kc else "N")
            self.other.append(((d.M, d.N, d.K), f"{lay} {kind}", 2.0 * d.M * d.N * d.K, a, b))
            return r
        self.rec.append(((d.M, d.N, d.K), kind, 2.0 * d.M * d.N * d.K, gemm_algo_bytes(d, e), a, b))
        return r

    def other_table(self, steps):
        shapes = {}
        for (mnk, kind, fl, a, b) in self.other:
            c = shapes.setdefault(f"{mnk[0]}x{mnk[1]}x{mnk[2]} {kind}", [0, 0.0, fl])
            c[0] += 1
            c[1] += a.elapsed_time(b)
        lines = [f"{v[1] / max(1, steps) * 1e3:9.1f} us/step {v[0] // max(1, steps):4d}x {1e3 * v[1] / v[0]:8.1f} us "
                 f"{v[2] / (v[1] / v[0] / 1e3) / 1e12:7.1f} TF/s  {k}" for k, v in sorted(shapes.items(), key=lambda kv: -kv[1][1])]
        tot = sum(v[1] for v in shapes.values()) / max(1, steps)
        return "\n".join(lines + [f"other GEMM launches (each alone, incl. split-K reduce): {tot:.3f} ms/step"])

    def summary(self, steps):
        tot_ms = sum(a.elapsed_time(b) for *_, a, b in self.rec)
        flops = sum(r[2] for r in self.rec)
        nbytes = sum(r[3] for r in self.rec)
        n = len(self.rec)
        shapes = {}
        for (mnk, kind, fl, _, a, b) in self.rec:
            k = f"{mnk[0]}x{mnk[1]}x{mnk[2]} {kind}"
            c = shapes.setdefault(k, [0, 0.0, fl])
            c[0] += 1
            c[1] += a.elapsed_time(b)
        per_shape = {k: {"launches_per_step": v[0] // max(1, steps), "mean_us": round(1e3 * v[1] / v[0], 1),
                         "tflops": round(v[2] / (v[1] / v[0] / 1e3) / 1e12, 1)} for k, v in shapes.items()}
        return {"launches": n, "launches_per_step": n // max(1, steps), "mean_launch_ms": tot_ms / max(1, n),
                "flop_per_launch": flops / max(1, n), "algo_bytes_per_launch": nbytes / max(1, n),
                "ms_per_step": tot_ms / max(1, steps), "per_shape": per_shape}


def pmc_traffic(timeout_s=240):
    """HBM bytes per launch of the roofline kernel (gemm_8ph_kernel) from rocprofv3 PMC counters,
    one counter per pass (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE in KiB; on gfx950
    FETCH_SIZE reads half the bytes of a 16 B/lane streaming read -- the GEMM's LDS-DMA operand
    loads -- so it is doubled; WRITE_SIZE is exact for 16 B/lane stores). Runs
    tools/traffic_probe.py (ViT-B/16 bs=256 train steps) as a CHILD process under rocprofv3
    before this process touches the GPU; averages every gemm_8ph dispatch of the run.
    Returns (bytes, detail) or (None, reason)."""
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
                if "gemm_8ph" in row.get("Kernel_Name", "") and row.get("Counter_Name", "") == ctr:
                    per.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not per:
            return None, f"{ctr}: no gemm_8ph dispatch in the counter CSV"
        vals[ctr] = (sum(per) / len(per), len(per))  # mean over the probe's launches (KiB)
    read_b = 2.0 * vals["FETCH_SIZE"][0] * 1024
    write_b = vals["WRITE_SIZE"][0] * 1024
    return read_b + write_b, {"read_bytes": round(read_b), "write_bytes": round(write_b),
                              "fetch_size_kib": vals["FETCH_SIZE"][0], "write_size_kib": vals["WRITE_SIZE"][0],
                              "dispatches": vals["FETCH_SIZE"][1],
                              "method": "rocprofv3 --pmc, one counter per pass, mean over every gemm_8ph dispatch "
                                        "of 2 ViT-B/16 bs=256 train steps (tools/traffic_probe.py); read = "
                                        "2*FETCH_SIZE (gfx950 16 B/lane correction)"}


def cpu_model() -> str:
    """Host CPU model name (/proc/cpuinfo, as `lscpu` reports it)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(cfg_name, budget_s=12.0, bs=None):
    """Oracle train step (fp32, torch CPU ops: oracle/vit_oracle.py, zero_grad -> fwd (dropout
    0.1) -> CE(ls 0.1) -> bwd -> AdamW as `train/train_image_vit.py:117-130`) on a bounded
    sample of the workload: `bs` images per step (default: the config's batch for small
    models, 2 for ViT-B), up to 20 timed steps within about budget_s."""
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
        for k, s_ in (("self_attn.in_proj_weight", (3 * D, D)), ("self_attn.out_proj.weight", (D, D)),
                      ("linear1.weight", (F, D)), ("linear2.weight", (D, F))):
            p[pre + k] = torch.randn(*s_, generator=g) * 0.02
        for k, s_ in (("self_attn.in_proj_bias", 3 * D), ("self_attn.out_proj.bias", D), ("linear1.bias", F),
                      ("linear2.bias", D), ("norm1.bias", D), ("norm2.bias", D)):
            p[pre + k] = torch.zeros(s_)
        p[pre + "norm1.weight"] = torch.ones(D)
        p[pre + "norm2.weight"] = torch.ones(D)
    for t in p.values():
        t.requires_grad_(True)
    m = {k: torch.zeros_like(v) for k, v in p.items()}
    v2 = {k: torch.zeros_like(v) for k, v in p.items()}
    if bs is None:
        bs = 2 if D >= 768 else B
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
    return {"value": round(bs / med, 3), "unit": "images/s", "cores": threads, "cpu_model": cpu_model(), "kind": "port",
            "sample": f"{cfg_name}: oracle train step (fwd+bwd+AdamW, fp32, dropout 0.1, CE ls 0.1) at bs={bs}, "
                      f"{len(times)} timed steps, median {med * 1e3:.0f} ms/step, torch {torch.__version__}"}


def spawn_ranks(args) -> int:
    """--gpus N > 1 outside torch.distributed: run this script under torch.distributed.run as a
    child process (this process never initialises the GPU) and relay its output."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    r = subprocess.run(cmd, env=env)
    return r.returncode


def percentile(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    i = min(len(xs) - 1, max(0, int(round(q * (len(xs) - 1)))))
    return xs[i]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="vit_base_224", choices=list(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--probe-steps", type=int, default=2, help="steps of the (untimed) roofline probe phase")
    ap.add_argument("--probe-all", action="store_true",
                    help="probe phase: time every other GEMM launch too (stderr table, not the JSON line)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the whole step as a HIP graph (auto: on for the launch-bound small configs)")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="N>1: dtype of the gradient all-reduce (bf16 halves the bytes; default fp32)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch plumbing only (gloo, CPU): ranks rendezvous, barrier, rank 0 prints the JSON line")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            dist.barrier()
            seen = dist.get_world_size()
            dist.destroy_process_group()
        else:
            seen = 1
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "images/s", "n_gpus": world,
                              "ranks_seen": seen, "dry_run": True}), flush=True)
        return

    traffic, traffic_detail = None, "not measured (N>1, --no-traffic or not the ViT-B/16 config)"
    if world == 1 and not args.no_traffic and args.config == "vit_base_224":
        # child rocprofv3 passes first: this process has not initialised the GPU yet
        traffic, traffic_detail = pmc_traffic()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    rccl = None
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
        try:
            v = torch.cuda.nccl.version()
            rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001
            rccl = "unknown"

    import fervit
    from fervit import ops, runtime

    fervit.manual_seed(1234 + rank)
    torch.manual_seed(42)
    model, opt, crit, B, shape, desc = build(args.config, device)
    net = model
    if world > 1:
        from fervit.ddp import DistributedDataParallel

        net = DistributedDataParallel(model, grad_dtype=torch.bfloat16 if args.grad_dtype == "bf16" else torch.float32)
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
    probe = GemmProbe(args.probe_all)
    ops.LAUNCH_PROBE = probe

    def step():
        opt.zero_grad()
        loss = crit(net(x), y)
        loss.backward()
        opt.step()
        return loss

    # (with N > 1 the captured step holds the RCCL bucket all-reduces too: fervit/ddp.py)
    use_graph = args.graph == "on" or (args.graph == "auto" and args.config != "vit_base_224")
    for _ in range(args.warmup):
        step()
    if use_graph:
        from fervit.graph import StepGraph

        graph = StepGraph(step, opt, warmup=1).capture()
        run = graph.replay
    else:
        run = step
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(args.steps):
        loss = run()
        ev[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    step_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    lossv = loss.item()
    # probe phases (untimed): HIP events around every gemm_8ph launch of a few eager steps.
    # In-step: as the timed steps run them (weight-gradient stream on, so a launch may share the chip
    # with a concurrent split-K weight gradient); isolated (the roofline `frac`): weight-gradient
    # stream off, every launch alone on the chip.
    if use_graph:
        graph.release()
    probe.on = True
    for _ in range(args.probe_steps):
        step()
    torch.cuda.synchronize()
    ps_in = probe.summary(args.probe_steps)
    probe.rec, probe.other = [], []
    wg_on = runtime.WGRAD.enabled
    runtime.WGRAD.enabled = False
    for _ in range(args.probe_steps):
        step()
    torch.cuda.synchronize()
    probe.on = False
    runtime.WGRAD.enabled = wg_on
    ps = probe.summary(args.probe_steps)
    if probe.all and rank == 0:
        print(probe.other_table(args.probe_steps), file=sys.stderr, flush=True)
    ms = el / args.steps * 1e3
    imgs = world * B * args.steps / el
    step_tflops = flops_img * B / (ms / 1e3) / 1e12
    achieved = ps["flop_per_launch"] / (ps["mean_launch_ms"] / 1e3) / 1e12 if ps["launches"] else 0.0
    achieved_in = ps_in["flop_per_launch"] / (ps_in["mean_launch_ms"] / 1e3) / 1e12 if ps_in["launches"] else 0.0
    if rank == 0:
        cpu = cpu1 = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.config)
            if args.config == "vit_base_224":
                cpu1 = cpu_baseline("image_vit_48", bs=64)
        out = {
            "metric": METRIC, "value": round(imgs, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (N(0,1) inputs, uniform labels), random init",
            "config": {"workload": desc, "per_gpu_batch": B, "global_batch": B * world, "tokens": N,
                       "parallelism": f"dp{world}", "grad_allreduce": args.grad_dtype if world > 1 else None},
            "step_ms_median": round(percentile(step_ms, 0.5), 3), "step_ms_p10": round(percentile(step_ms, 0.1), 3),
            "step_ms_p90": round(percentile(step_ms, 0.9), 3),
            "roofline": {"bound": "mfma", "kernel": "gemm_8ph_kernel (bf16 MFMA; every fwd + dgrad linear and the "
                                                    "patch embed, fused epilogues)",
                         "achieved": round(achieved, 1), "peak": round(PEAK_BF16_TFLOPS, 1), "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                         "frac_in_step": round(achieved_in / PEAK_BF16_TFLOPS, 4),
                         "mean_launch_ms_in_step": round(ps_in["mean_launch_ms"], 4),
                         "frac_note": "frac: each launch alone on the chip (weight-gradient stream off); "
                                      "frac_in_step: the same launches in eager train steps with the "
                                      "weight-gradient stream on (sharing CUs with split-K weight gradients)",
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_detail": traffic_detail,
                         "algorithmic_bytes": round(ps["algo_bytes_per_launch"]),
                         "flop_per_launch": round(ps["flop_per_launch"]),
                         "launches_per_step": ps["launches_per_step"],
                         "mean_launch_ms": round(ps["mean_launch_ms"], 4),
                         "kernel_ms_per_step": round(ps["ms_per_step"], 3),
                         "per_shape": ps["per_shape"]},
            "launch": "hipGraph replay of the whole step" if use_graph else "eager (one host launch per kernel)",
            "step_mfma_frac": round(step_tflops / PEAK_BF16_TFLOPS, 4),
            "step_tflops": round(step_tflops, 1),
            "final_loss": round(lossv, 4),
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "rccl": rccl,
            "cpu_baseline": cpu,
            "cpu_baseline_cfg1": cpu1,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
