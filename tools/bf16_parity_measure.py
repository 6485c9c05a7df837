"""Measure the bf16 production path's errors against the reference fixtures (and, at the headline
size, against this library's fp32 parity path) -- the numbers tests/test_gpu_models.py pins its
bf16 gates to (2x measured). Prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fer-vit_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cases import CASES, case_inputs  # noqa: E402
from test_gpu_models import build  # noqa: E402


def fixture_errors(name):
    m, fx = build(name)
    m.set_precision("bf16").train()
    x, y = case_inputs(name)
    logits = m(x.cuda())
    torch.nn.functional.cross_entropy(logits, y.cuda(), label_smoothing=0.1).backward()
    lg = logits.detach().cpu().numpy()
    ref = fx["logits"]
    params = dict(m.named_parameters())
    gn, gs = 0.0, 0.0
    for k, gl2, samp, idx in zip(fx["grad_keys"], fx["grad_l2"], fx["grad_samples"], fx["grad_idx"]):
        g = params[str(k)].grad.detach().reshape(-1).double().cpu()
        gn = max(gn, abs(g.norm().item() - gl2) / (gl2 + 1e-12))
        ok = idx >= 0
        if ok.any():
            gs = max(gs, float(np.abs(g[idx[ok]].numpy() - samp[ok]).max()) / (gl2 + 1e-12))
    return {"logits_abs": float(np.abs(lg - ref).max()), "ref_absmax": float(np.abs(ref).max()),
            "grad_norm_rel": gn, "grad_sample_rel": gs}


def headline():
    from models_fer_vit.image_vit import create_vit_base

    torch.manual_seed(0)
    m = create_vit_base(num_classes=7, img_size=224).cuda()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(256, 3, 224, 224, generator=g).cuda()
    out = {}
    with torch.no_grad():
        for prec in ("fp32", "bf16"):
            m.set_precision(prec).eval()
            out[prec] = m(x).float().cpu()
    a, b = out["fp32"], out["bf16"]
    top2 = a.topk(2, dim=1).values
    margin = top2[:, 0] - top2[:, 1]
    sure = margin > 0.2
    return {"logits_abs": float((a - b).abs().max()), "ref_absmax": float(a.abs().max()),
            "argmax_equal_sure": bool((a.argmax(1)[sure] == b.argmax(1)[sure]).all()),
            "n_sure": int(sure.sum()), "n": int(a.shape[0])}


if __name__ == "__main__":
    res = {name: fixture_errors(name) for name in CASES}
    res["vit_base_224_bs256_vs_fp32"] = headline()
    print(json.dumps(res, indent=1))
