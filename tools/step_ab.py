"""Interleaved step-time A/B of run-time variants in ONE process (cdna_hip_programming.md rule 24).

    python tools/step_ab.py --config vit_base_224 --rounds 4 --steps 10 base wg:m8lt6 wg:lt192 ...

The model (bench.py build) is built once; every round runs each variant for --steps timed train
steps (after one untimed step) and records the mean step time; the table gives the median and min
over rounds. Variants:
  base           as shipped (bench.py: the step on the legacy null stream)
  nb:<variant>   the variant with the step on a non-blocking stream (every variant below does that)
  wg:<pred>      weight-gradient side stream restricted to the CUs whose mask bit satisfies <pred>
  cs:<pred>      the whole step issued on a CU-masked compute stream (weight gradients unmasked)
  both:<p1>/<p2> compute stream on <p1>, weight-gradient stream on <p2>
  wgoff          weight gradients on the compute stream
  adamwbw        FusedAdamW.step_in_backward (per-layer updates from the backward's gradient-ready hook)
  noadamcache    FusedAdamW uploads its segment table every step (the round-4 behaviour)
  lib:<k>=<v>    a library selector for the variant: attnfwd (fer_attention_set_fwd_kernel), gemmcfg
  env:<N>=<v>    environment variable N set to v for the variant (for switches the library reads per call)
  hp             the step on a high-priority non-blocking stream (torch priority -1), weight gradients at the
                 default priority (compare with nb:base)
  hpwg           the opposite: the weight-gradient stream at high priority, the step on nb:base's stream
<pred>: lt<N> (bit < N), ge<N> (bit >= N), m<K>lt<N> (bit % K < N), m<K>ge<N> (bit % K >= N).
"""
import argparse
import ctypes
import os
import re
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))

import torch  # noqa: E402


def mask_words(pred: str, ncu: int):
    m = re.fullmatch(r"(lt|ge)(\d+)", pred)
    if m:
        op, n = m.group(1), int(m.group(2))
        f = (lambda i: i < n) if op == "lt" else (lambda i: i >= n)
    else:
        m = re.fullmatch(r"m(\d+)(lt|ge)(\d+)", pred)
        if not m:
            raise SystemExit(f"bad mask predicate {pred}")
        k, op, n = int(m.group(1)), m.group(2), int(m.group(3))
        f = (lambda i: i % k < n) if op == "lt" else (lambda i: i % k >= n)
    words = [0] * ((ncu + 31) // 32)
    for i in range(ncu):
        if f(i):
            words[i // 32] |= 1 << (i % 32)
    return words


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="vit_base_224")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()

    import bench
    from fervit import runtime
    from fervit._lib import check, lib

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    torch.manual_seed(42)
    model, opt, crit, B, shape, desc = bench.build(a.config, dev)
    g = torch.Generator(device=dev).manual_seed(42)
    x = torch.randn(B, *shape, device=dev, generator=g)
    y = torch.randint(0, 7, (B,), device=dev, generator=g)

    def step():
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        opt.step()
        return loss

    # Streams are created once per CU mask and never destroyed (the caching allocator keeps events of
    # the streams its blocks were used on), and every variant after "base" issues its step on a
    # non-blocking compute stream: hipExtStreamCreateWithCUMask streams are BLOCKING streams, which
    # synchronise with the legacy null stream bench.py's step runs on.
    streams = {}

    def masked(pred):
        if pred not in streams:
            words = mask_words(pred, ncu)
            arr = (ctypes.c_uint32 * len(words))(*words)
            h = ctypes.c_void_p()
            check(lib().fer_stream_create_cu_mask(arr, len(words), 0, ctypes.byref(h)), "masked stream")
            streams[pred] = torch.cuda.ExternalStream(h.value, device=dev)
        return streams[pred]

    nb_compute = torch.cuda.Stream(device=dev)
    hp_compute = torch.cuda.Stream(device=dev, priority=-1)
    hp_side = torch.cuda.Stream(device=dev, priority=-1)
    print("stream priority range", torch.cuda.Stream.priority_range(), flush=True)
    default_side = {}

    def setup(v):
        lib().fer_attention_set_fwd_kernel(0)
        lib().fer_gemm_set_config(-1)
        opt.step_in_backward(False)
        opt.cache_table = True
        runtime.WGRAD.enabled = True
        if "side" not in default_side:  # the shipped side stream (created by the first backward)
            default_side["side"] = runtime.WGRAD.streams.get(dev)
        runtime.WGRAD.streams[dev] = default_side["side"]
        if runtime.WGRAD.streams[dev] is None:
            del runtime.WGRAD.streams[dev]
        for k in [k for k in os.environ if k.startswith("FERVIT_AB_")]:
            del os.environ[k[len("FERVIT_AB_"):]]
            del os.environ[k]
        if v == "base":
            return None
        if v.startswith("env:"):  # env:NAME=VALUE, read by the library at each call (on the null stream, as base)
            name, val = v[4:].split("=", 1)
            os.environ[name] = val
            os.environ["FERVIT_AB_" + name] = "1"  # (undone by the next setup)
            return None
        cs = nb_compute
        body = v[3:] if v.startswith("nb:") else v
        if body == "base":
            pass
        elif body == "wgoff":
            runtime.WGRAD.enabled = False
        elif body == "hp":
            cs = hp_compute
        elif body == "hpwg":
            runtime.WGRAD.streams[dev] = hp_side
        elif body == "adamwbw":  # optimizer step inside the backward (FusedAdamW.step_in_backward)
            opt.step_in_backward(True)
        elif body == "noadamcache":  # FusedAdamW re-uploads its segment table every step (round-4 behaviour)
            opt.cache_table = False
        elif body.startswith("lib:"):  # a library run-time selector, e.g. lib:attnfwd=2
            k, val = body[4:].split("=")
            fn = {"attnfwd": "fer_attention_set_fwd_kernel", "gemmcfg": "fer_gemm_set_config"}[k]
            check(getattr(lib(), fn)(int(val)), fn)
        elif body.startswith("wg:"):
            runtime.WGRAD.streams[dev] = masked(body[3:])
        elif body.startswith("cs:"):
            cs = masked(body[3:])
        elif body.startswith("both:"):
            p1, p2 = body[5:].split("/")
            cs = masked(p1)
            runtime.WGRAD.streams[dev] = masked(p2)
        else:
            raise SystemExit(f"unknown variant {v}")
        return cs

    def timed(v, n):
        cs = setup(v)
        ctx = torch.cuda.stream(cs) if cs is not None else torch.cuda.stream(torch.cuda.current_stream(dev))
        with ctx:
            if cs is not None:
                cs.wait_stream(torch.cuda.default_stream(dev))
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                loss = step()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, loss.item()

    for v in a.variants:
        timed(v, a.warmup)
    res = {v: [] for v in a.variants}
    for r in range(a.rounds):
        for v in a.variants:
            ms, lv = timed(v, a.steps)
            res[v].append(ms)
            print(f"round {r} {v:24s} {ms:8.3f} ms  loss {lv:.4f}", flush=True)
    print(f"\n{a.config}: {a.rounds} rounds x {a.steps} steps per variant (ms/step)")
    for v in a.variants:
        xs = res[v]
        print(f"  {v:24s} median {statistics.median(xs):8.3f}  min {min(xs):8.3f}  max {max(xs):8.3f}")


if __name__ == "__main__":
    main()
