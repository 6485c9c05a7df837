"""Host-side pieces of the trainers' step functions (fer-vit_amd/train): class weights
(`train/train_image_vit.py:82-107` formula), once-per-epoch metrics equal to sklearn on the
same predictions, and the layer-wise optimizer groups (`train_hybrid_latent_vit.py:63-117`)."""
import numpy as np
import torch

from train.common import EpochStats, calculate_class_weights, layerwise_param_groups


def test_class_weights_formula():
    y = torch.tensor([0, 0, 1, 2, 2, 2, 3, 3, 4, 5, 6, 6])
    ds = torch.utils.data.TensorDataset(torch.zeros(len(y), 2), y)
    w = calculate_class_weights(ds)
    counts = np.bincount(y.numpy(), minlength=7)
    assert torch.allclose(w, torch.tensor(len(y) / (7 * counts), dtype=torch.float32))
    sub = torch.utils.data.Subset(ds, [0, 1, 2, 3])
    w2 = calculate_class_weights(sub)  # classes {0: 2, 1: 1, 2: 1} -> 3 classes
    assert torch.allclose(w2, torch.tensor([4 / 6, 4 / 3, 4 / 3]))


def test_epoch_stats_match_sklearn():
    from sklearn.metrics import accuracy_score, f1_score

    g = torch.Generator().manual_seed(0)
    st = EpochStats("cpu")
    allp, ally = [], []
    for _ in range(5):
        logits = torch.randn(16, 7, generator=g)
        y = torch.randint(0, 7, (16,), generator=g)
        st.add(torch.tensor(0.5), 16, logits, y)
        allp.extend(logits.argmax(1).tolist())
        ally.extend(y.tolist())
    r = st.finish(80)
    assert abs(r["loss"] - 0.5) < 1e-12
    assert r["accuracy"] == accuracy_score(ally, allp)
    assert r["f1_macro"] == f1_score(ally, allp, average="macro")
    assert r["f1_weighted"] == f1_score(ally, allp, average="weighted")


def test_layerwise_groups():
    class V(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.input_proj = torch.nn.Linear(4, 4)
            self.transformer = torch.nn.ModuleList([torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)])
            self.transformer[0].weight.requires_grad_(False)
            self.use_adapter = True
            self.adapters = torch.nn.ModuleList([torch.nn.Linear(4, 2)])
            self.head = torch.nn.Linear(4, 7)
            self.pos_embed = torch.nn.Parameter(torch.zeros(1, 3, 4))
            self.cls_token = torch.nn.Parameter(torch.zeros(1, 1, 4))

    v = V()
    gs = layerwise_param_groups(v, 1e-3, 0.05, log=lambda *_: None)
    assert [g["lr"] for g in gs] == [1e-2, 1e-3, 1e-2, 1e-2, 5e-3]
    assert len(gs[1]["params"]) == 3 and gs[-1]["weight_decay"] == 0
