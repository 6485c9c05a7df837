"""Generate the committed golden fixtures by running the REFERENCE model code.

Run once, in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
It imports the reference's torch-only model files, loads deterministic weights
(`detparams.py`, keyed by state_dict name), runs a train-mode forward (dropout
constructed as 0.0 so RNG streams do not matter), CrossEntropyLoss with
label smoothing 0.1, backward, and one AdamW step (lr 1e-3, wd 0.05), and writes
small `.npz` fixtures: logits, loss, per-parameter gradient {sum, L2, 8 samples},
post-AdamW parameter samples, and eval-mode logits (the reference's fused
inference path). Nothing from the reference is copied into the repo; only these
numeric vectors are. The GPU box never runs this script.
"""
from __future__ import annotations

import os
import sys
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from detparams import det_directions, det_input, det_labels, det_state_dict  # noqa: E402

REF = "/root/reference"


def sample_idx(key: str, numel: int, k: int = 8) -> np.ndarray:
    g = np.random.default_rng(zlib.crc32(("idx:" + key).encode()))
    return np.sort(g.choice(numel, size=min(k, numel), replace=False))


def load_det(model: torch.nn.Module, seed: int = 0) -> None:
    sd = model.state_dict()
    det = det_state_dict([(k, tuple(v.shape)) for k, v in sd.items()], seed)
    model.load_state_dict(det)


def run_case(name: str, model: torch.nn.Module, x: torch.Tensor, labels: torch.Tensor, out: dict,
             ls: float = 0.1) -> None:
    torch.manual_seed(0)
    load_det(model)
    model.train()
    logits = model(x)
    loss = torch.nn.CrossEntropyLoss(label_smoothing=ls)(logits, labels)
    loss.backward()
    rec = {"logits": logits.detach().numpy(), "loss": np.float64(loss.item()), "labels": labels.numpy()}
    sd = model.state_dict()
    rec["sd_keys"] = np.array(list(sd.keys()))
    rec["sd_shapes"] = np.array([",".join(str(d) for d in v.shape) for v in sd.values()])
    top = torch.topk(logits.detach(), 2, dim=1).values
    rec["margin"] = (top[:, 0] - top[:, 1]).numpy()
    keys, gsum, gl2, gsamp, gidx = [], [], [], [], []
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().reshape(-1).double()
        idx = sample_idx(k, g.numel())
        keys.append(k)
        gsum.append(g.sum().item())
        gl2.append(g.norm().item())
        s = np.full(8, np.nan)
        s[: len(idx)] = g[idx].numpy()
        gsamp.append(s)
        ii = np.full(8, -1, np.int64)
        ii[: len(idx)] = idx
        gidx.append(ii)
    rec.update(grad_keys=np.array(keys), grad_sum=np.array(gsum), grad_l2=np.array(gl2),
               grad_samples=np.array(gsamp), grad_idx=np.array(gidx))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=0.05)
    opt.step()
    psamp = []
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        idx = sample_idx(k, p.numel())
        s = np.full(8, np.nan)
        s[: len(idx)] = p.detach().reshape(-1)[idx].double().numpy()
        psamp.append(s)
    rec["adamw_samples"] = np.array(psamp)
    load_det(model)
    model.eval()
    with torch.no_grad():
        rec["logits_eval"] = model(x).numpy()
    out[name] = rec
    print(f"{name}: loss={rec['loss']:.6f} logits[0]={rec['logits'][0][:3]} min-margin={rec['margin'].min():.3g}")


def pick_rows(model: torch.nn.Module, name: str, shape, need: int, min_margin: float = 1e-2):
    """SURVEY §7 fixture rule: keep only samples whose top-1 / top-2 logit margin is >= 1e-2, so
    argmax equality is well posed. Draws a pool of 3x `need` deterministic inputs, runs the
    reference forward (train mode, dropout 0: per-sample, no batch coupling) and returns the
    first `need` rows that pass (their pool indices are stored in the fixture)."""
    pool = det_input(name, (3 * need,) + tuple(shape[1:]))
    load_det(model)
    model.train()
    with torch.no_grad():
        lg = model(pool)
    top = torch.topk(lg, 2, dim=1).values
    ok = ((top[:, 0] - top[:, 1]) >= min_margin).nonzero().flatten()[:need]
    assert ok.numel() == need, f"{name}: only {ok.numel()} samples pass the margin rule"
    labels = det_labels(name, 3 * need)[ok]
    return pool[ok], labels, ok.numpy()


def adapter_case(out: dict) -> None:
    """AdapterModule (`hybrid_latent_vit.py:249-265`) at the cfg4 geometry (768 -> 64 -> 768),
    det weights, x [4,19,768]; forward, and backward of sum(y * dy) for det dy."""
    from models_fer_vit.hybrid_latent_vit import AdapterModule

    m = AdapterModule(768, 64)
    load_det(m)
    with torch.no_grad():
        m.alpha.fill_(0.37)  # away from the init so the residual branch carries weight
    x = det_input("adapter_x", (4, 19, 768)).requires_grad_(True)
    dy = det_input("adapter_dy", (4, 19, 768))
    y = m(x)
    (y * dy).sum().backward()
    rec = {"alpha": np.float32(0.37)}
    tensors = {"y": y.detach(), "dx": x.grad}
    tensors.update({"grad:" + k: p.grad for k, p in m.named_parameters()})
    for k, t in tensors.items():
        put_summary(rec, k, t)
    out["adapter"] = rec
    print("adapter: |y|", float(y.detach().norm()))


def pos_interp_case(out: dict) -> None:
    """HybridLatentViT._init_position_embedding (`hybrid_latent_vit.py:118-156`) on a det
    ViT-B pos_embed [1,197,768]: seq_len 18 (w+), 36 (concat decomposer) and 196 (no interp).
    The method only reads `pretrained_vit.pos_embed` (and self.embed_dim when there is none)."""
    import types

    from models_fer_vit.hybrid_latent_vit import HybridLatentViT

    pe = torch.nn.Parameter(det_input("pos_embed_vitb", (1, 197, 768)))
    stub = types.SimpleNamespace(pos_embed=pe)
    me = types.SimpleNamespace(embed_dim=768)
    rec = {}
    for L in (18, 36, 196):
        r = HybridLatentViT._init_position_embedding(me, stub, L).detach()
        rec[f"L{L}:shape"] = np.array(r.shape)
        if L < 196:
            rec[f"L{L}"] = r[0, :, :64].numpy().copy()  # every position, first 64 channels
        put_summary(rec, f"L{L}", r)
    out["pos_interp"] = rec


def put_summary(rec: dict, key: str, t: torch.Tensor, k: int = 256) -> None:
    """Large tensors go in as {sum, L2, k fixed-index samples} (fixtures stay small)."""
    f = t.detach().reshape(-1).double()
    idx = sample_idx(key, f.numel(), k)
    rec[key + ":sum"] = np.float64(f.sum().item())
    rec[key + ":l2"] = np.float64(f.norm().item())
    rec[key + ":idx"] = idx
    rec[key + ":samples"] = f[idx].numpy()


def main() -> None:
    only = set(sys.argv[1:])
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    from models_fer_vit.image_vit import ImageViT
    from models_fer_vit.latent_vit import LatentViT
    from models_fer_vit.latent_vit_v2 import LatentViTv2
    from models_fer_vit.latent_decomposer import LatentDecomposer

    cases = {}
    # cfg1 shape: ImageViT d6/h8 e384 on 48x48 (BASELINE configs[0])
    m = ImageViT(img_size=48, patch_size=16, in_channels=3, embed_dim=384, depth=6, heads=8,
                 mlp_dim=1536, num_classes=7, dropout=0.0)
    run_case("image_vit_48", m, det_input("image_vit_48", (8, 3, 48, 48)), det_labels("image_vit_48", 8), cases)
    # ViT-B/16 224 (BASELINE configs[2]) at B=2
    m = ImageViT(img_size=224, patch_size=16, in_channels=3, embed_dim=768, depth=12, heads=12,
                 mlp_dim=3072, num_classes=7, dropout=0.0)
    run_case("vit_base_224", m, det_input("vit_base_224", (2, 3, 224, 224)), det_labels("vit_base_224", 2), cases)
    # LatentViT defaults (configs[1])
    m = LatentViT(dropout=0.0)
    run_case("latent_vit", m, det_input("latent_vit", (8, 18, 512)), det_labels("latent_vit", 8), cases)
    # LatentViTv2 with every prologue flag
    m = LatentViTv2(dropout=0.0, use_lwn=True, use_lwn_residual=True, use_spe=True, use_leam=True)
    xs, ys, rows = pick_rows(m, "latent_vit_v2_all", (8, 18, 512), 8)
    run_case("latent_vit_v2_all", m, xs, ys, cases)
    cases["latent_vit_v2_all"]["input_rows"] = rows
    # LatentViTv2, LWN without residual gate, + LEAM, small depth/heads variant
    m = LatentViTv2(dropout=0.0, depth=2, heads=4, mlp_dim=1024, use_lwn=True, use_leam=True)
    run_case("latent_vit_v2_lwn", m, det_input("latent_vit_v2_lwn", (4, 18, 512)),
             det_labels("latent_vit_v2_lwn", 4), cases)

    # LatentDecomposer, every output/decompose mode (fixtures for a14)
    dirs = det_directions(7, 18, 512)
    dec = LatentDecomposer({i: dirs[i] for i in range(7)}, 18, 512)
    w = det_input("decomposer", (4, 18, 512))
    drec = {"directions_buffer_sum": np.float64(dec.directions.double().sum().item())}
    for dm in ("all_classes", "max_class"):
        for om in ("expr_only", "id_only", "enhanced", "concat"):
            with torch.no_grad():
                y = dec(w, output_mode=om, enhance_alpha=2.0, decompose_mode=dm)
            yf = y.reshape(-1).double()
            idx = sample_idx(f"dec:{dm}:{om}", yf.numel(), 64)
            drec[f"{dm}:{om}:shape"] = np.array(y.shape)
            drec[f"{dm}:{om}:sum"] = np.float64(yf.sum().item())
            drec[f"{dm}:{om}:l2"] = np.float64(yf.norm().item())
            drec[f"{dm}:{om}:idx"] = idx
            drec[f"{dm}:{om}:samples"] = yf[idx].numpy()
        with torch.no_grad():
            drec[f"{dm}:scores"] = dec.get_expression_scores(w).numpy()
    cases["decomposer"] = drec
    adapter_case(cases)
    pos_interp_case(cases)

    for name, rec in cases.items():
        if only and name not in only:
            continue
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    print("wrote", len(cases), "fixtures")


if __name__ == "__main__":
    main()
