"""Packed w+ shards (fervit.data, libfervit_io.so) on the CPU: the shard holds exactly the
samples of a reference-format latent directory (`data/generate_latents.py:87-91` files,
`data/latent_dataset.py` order), the native gather is bit-exact in any index order, and the
loader's epoch order / rank split behave like a shuffled DistributedSampler."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make_dir(path, n=37, L=18, D=512, seed=0):
    g = torch.Generator().manual_seed(seed)
    os.makedirs(path, exist_ok=True)
    order = torch.randperm(n, generator=g).tolist()  # creation order != sorted order
    ref = {}
    for i in order:
        lat = torch.randn(L, D, generator=g)
        lab = int(torch.randint(0, 7, (1,), generator=g))
        torch.save({"latent": lat, "label": lab, "img_path": f"/data/fer/{i:05d}.png"},
                   os.path.join(path, f"{i:05d}.pt"))
        ref[i] = (lat, lab)
    return [ref[i] for i in range(n)]  # sorted-name order == i order


@pytest.fixture(scope="module")
def shard(tmp_path_factory):
    from fervit.data import pack_latent_dir

    d = tmp_path_factory.mktemp("latents")
    ref = _make_dir(str(d / "train"))
    out = str(d / "train.fwps")
    assert pack_latent_dir(str(d / "train"), out) == len(ref)
    return out, ref


def test_shard_holds_every_sample_in_reference_order(shard):
    from fervit.data import PackedLatentDataset

    path, ref = shard
    ds = PackedLatentDataset(path)
    assert len(ds) == len(ref) and (ds.L, ds.D) == (18, 512)
    for i, (lat, lab) in enumerate(ref):
        x, y = ds[i]
        assert torch.equal(x, lat) and y == lab
    assert ds.img_paths()[3] == "/data/fer/00003.png"
    counts = {}
    for _, lab in ref:
        counts[lab] = counts.get(lab, 0) + 1
    assert ds.get_class_counts() == counts
    assert ds.get_class_names()[3] == "happy"


def test_native_gather_any_order_bit_exact(shard):
    from fervit.data import PackedLatentDataset

    path, ref = shard
    ds = PackedLatentDataset(path)
    idx = np.random.default_rng(1).permutation(len(ref))[:29]
    out = torch.empty(len(idx), 18, 512)
    labs = np.empty(len(idx), dtype=np.int32)
    ds.gather(idx, out, labs, threads=4)
    for j, i in enumerate(idx):
        assert torch.equal(out[j], ref[i][0]) and labs[j] == ref[i][1]
    with pytest.raises(RuntimeError, match="out of range"):
        ds.gather(np.array([len(ref)]), out)


def test_corrupt_shard_is_rejected(tmp_path):
    from fervit.data import PackedLatentDataset

    bad = tmp_path / "bad.fwps"
    bad.write_bytes(b"NOTSHARD" + bytes(4096))
    with pytest.raises(RuntimeError, match="bad shard header"):
        PackedLatentDataset(str(bad))


def test_loader_epoch_order_and_rank_split(shard):
    from fervit.data import PackedLatentDataset, PackedLatentLoader

    path, ref = shard
    ds = PackedLatentDataset(path)
    ld = PackedLatentLoader(ds, batch_size=8, shuffle=True, seed=5, device=None)
    xs, ys = zip(*list(ld))
    x, y = torch.cat(xs), torch.cat(ys)
    assert x.shape == (len(ref), 18, 512)
    perm = np.random.default_rng(5).permutation(len(ref))
    for j, i in enumerate(perm):
        assert torch.equal(x[j], ref[i][0]) and int(y[j]) == ref[i][1]
    # the next epoch draws another permutation
    x2 = torch.cat([b for b, _ in ld])
    assert not torch.equal(x2, x)
    # two ranks: disjoint halves (padded), every sample covered, drop_last trims
    seen = []
    for r in range(2):
        lr = PackedLatentLoader(ds, batch_size=4, shuffle=True, seed=9, device=None, rank=r, world_size=2,
                                drop_last=True)
        n = sum(b.shape[0] for b, _ in lr)
        assert n == (len(ref) + 1) // 2 // 4 * 4
        lr2 = PackedLatentLoader(ds, batch_size=4, shuffle=True, seed=9, device=None, rank=r, world_size=2)
        seen.append(torch.cat([b for b, _ in lr2]))
    allx = torch.cat(seen)
    assert allx.shape[0] == len(ref) + 1
    keys = {tuple(a[0, :4].tolist()) for a in allx}
    assert keys == {tuple(lat[0, :4].tolist()) for lat, _ in ref}


def test_io_header_symbols_exported():
    import ctypes

    from fervit.data import IO_LIB_PATH

    src = open(os.path.join(ROOT, "include", "fervit_io.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = sorted(set(re.findall(r"\b(fio_[a-z_]+)\s*\(", src)))
    lib = ctypes.CDLL(IO_LIB_PATH)
    assert names and all(hasattr(lib, n) for n in names), names
