"""Packed-shard loader into HBM and the on-device LatentAugment (`data/latent_dataset.py:6-49`).

The loader's device batches equal the host samples (bit-exact); the augmentation matches the
reference transform's distributions: additive N(0, noise_std), one U(lo, hi) scale per sample,
feature mask with P(zero) = mask_prob (statistical checks: the reference draws from torch's RNG
stream, this from a counter hash, so only the distributions can agree)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_loader_device_batches_equal_host(tmp_path):
    from fervit.data import PackedLatentDataset, PackedLatentLoader, write_shard

    rng = np.random.default_rng(0)
    lat = rng.standard_normal((300, 18, 512), dtype=np.float32)
    lab = rng.integers(0, 7, 300)
    write_shard(str(tmp_path / "s.fwps"), lat, lab)
    ds = PackedLatentDataset(str(tmp_path / "s.fwps"))
    ld = PackedLatentLoader(ds, batch_size=64, shuffle=True, seed=3, device="cuda")
    perm = np.random.default_rng(3).permutation(300)
    got = 0
    for x, y in ld:
        assert x.is_cuda and x.dtype == torch.float32 and y.dtype == torch.int64
        idx = perm[got:got + x.shape[0]]
        assert torch.equal(x.cpu(), torch.from_numpy(lat[idx]))
        assert torch.equal(y.cpu(), torch.from_numpy(lab[idx]).long())
        got += x.shape[0]
    assert got == 300


def test_latent_augment_distributions():
    from fervit import ops
    from fervit._lib import check, lib

    B, LD = 512, 18 * 512
    z = torch.zeros(B, LD, device="cuda")
    check(lib().fer_latent_augment(z.data_ptr(), B, LD, 0.5, 1.0, 1.0, 0.0, 11, ops.stream()), "aug")
    assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 0.5) < 5e-3
    o = torch.ones(B, LD, device="cuda")
    check(lib().fer_latent_augment(o.data_ptr(), B, LD, 0.0, 0.9, 1.1, 0.0, 12, ops.stream()), "aug")
    s = o[:, 0]
    assert torch.equal(o, s[:, None].expand_as(o)) and s.min() >= 0.9 and s.max() <= 1.1
    assert abs(s.mean().item() - 1.0) < 0.01 and s.std().item() > 0.04
    m = torch.ones(B, LD, device="cuda")
    check(lib().fer_latent_augment(m.data_ptr(), B, LD, 0.0, 1.0, 1.0, 0.1, 13, ops.stream()), "aug")
    assert abs((m == 0).float().mean().item() - 0.1) < 2e-3 and torch.all((m == 0) | (m == 1))
