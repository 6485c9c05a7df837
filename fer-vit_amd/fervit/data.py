"""Packed w+ latent shards and a loader that feeds HBM.

The reference's latent trainers read one torch-pickled file per sample
(`data/latent_dataset.py:52-116`: LatentFERDataset, `torch.load` in `__getitem__`) through a
4-worker DataLoader (`train/train_latent_vit_v2.py:216-219`). At tens of thousands of images/s
per GPU that is the bottleneck, so here:

  * `pack_latent_dir(latent_dir, out)` writes every `.pt` sample of a directory -- in the
    reference's order (sorted file names, `latent_dataset.py:79-82`) -- into one shard file
    (format: csrc/io/latent_shard.cpp);
  * `PackedLatentDataset(path, transform)` is the drop-in Dataset: same `__getitem__`
    -> (latent fp32 [L, D], label), `get_class_counts`, `get_class_names`, backed by the
    native memory-mapped reader (`libfervit_io.so`, include/fervit_io.h);
  * `PackedLatentLoader` yields device batches: a background thread gathers batch k+1 with
    native threads into pinned memory while the GPU runs batch k, the H2D copy runs on a side
    stream, and LatentAugment (noise / per-sample scale / feature mask) runs on device
    (`fer_latent_augment`) instead of per sample on the host.
"""
from __future__ import annotations

import ctypes as C
import os
import queue
import threading
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
IO_LIB_PATH = os.environ.get("FERVIT_IO_LIB", os.path.join(_HERE, "libfervit_io.so"))
MAGIC = b"FWPS0001"
CLASS_NAMES = {0: "angry", 1: "disgust", 2: "fear", 3: "happy", 4: "neutral", 5: "sad", 6: "surprise"}

_io = None


def iolib():
    """ctypes binding of libfervit_io.so (raises if it is not built)."""
    global _io
    if _io is None:
        if not os.path.exists(IO_LIB_PATH):
            raise RuntimeError(f"fervit: {IO_LIB_PATH} missing -- build with `python __graft_entry__.py`")
        L = C.CDLL(IO_LIB_PATH)
        L.fio_open.restype, L.fio_open.argtypes = C.c_void_p, [C.c_char_p]
        L.fio_info.restype, L.fio_info.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int),
                                                            C.POINTER(C.c_int)]
        L.fio_labels.restype, L.fio_labels.argtypes = C.POINTER(C.c_int32), [C.c_void_p]
        L.fio_paths.restype, L.fio_paths.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_void_p),
                                                              C.POINTER(C.c_int64)]
        L.fio_gather.restype, L.fio_gather.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                                                C.c_void_p, C.c_int]
        L.fio_close.restype, L.fio_close.argtypes = None, [C.c_void_p]
        L.fio_last_error.restype, L.fio_last_error.argtypes = C.c_char_p, []
        _io = L
    return _io


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: {iolib().fio_last_error().decode()}")


# ------------------------------------------------------------------ writer
def pack_latent_dir(latent_dir: str, out_path: str) -> int:
    """Pack every `*.pt` sample ({"latent": [L, D], "label": int, "img_path": str}, the file
    written by `data/generate_latents.py:87-91`) of `latent_dir`, in sorted file-name order,
    into one shard. Files are read with `torch.load(weights_only=True)`. Returns the count."""
    if not os.path.isdir(latent_dir):
        raise FileNotFoundError(f"Latent directory not found: {latent_dir}")
    files = sorted(f for f in os.listdir(latent_dir) if f.endswith(".pt"))
    if not files:
        raise ValueError(f"No .pt files found in {latent_dir}")
    first = torch.load(os.path.join(latent_dir, files[0]), map_location="cpu", weights_only=True)["latent"]
    Lx, Dx = int(first.shape[-2]), int(first.shape[-1])
    n = len(files)
    labels_off = 64
    latents_off = (labels_off + 4 * n + 4095) // 4096 * 4096
    paths = []
    tmp = out_path + ".tmp"
    with open(tmp, "wb") as f:
        f.truncate(latents_off + n * Lx * Dx * 4)
    mm = np.memmap(tmp, dtype=np.uint8, mode="r+")
    lab = np.ndarray((n,), dtype=np.int32, buffer=mm, offset=labels_off)
    lat = np.ndarray((n, Lx, Dx), dtype=np.float32, buffer=mm, offset=latents_off)
    for i, fn in enumerate(files):
        path = os.path.join(latent_dir, fn)
        try:
            d = torch.load(path, map_location="cpu", weights_only=True)
            x = d["latent"].float().reshape(-1, Dx)
            if x.shape != (Lx, Dx):
                raise ValueError(f"latent shape {tuple(d['latent'].shape)} != ({Lx}, {Dx})")
            lat[i] = x.numpy()
            lab[i] = int(d["label"])
            paths.append(str(d.get("img_path", "")))
        except Exception as e:  # the reference raises on a corrupt file too (latent_dataset.py:114-116)
            del mm
            os.remove(tmp)
            raise RuntimeError(f"Error loading {path}: {e}") from e
    mm.flush()
    del lab, lat, mm
    blob = b"\0".join(p.encode() for p in paths)
    paths_off = latents_off + n * Lx * Dx * 4
    with open(tmp, "r+b") as f:
        f.seek(paths_off)
        f.write(blob)
        f.seek(0)
        hdr = MAGIC + np.array([n], dtype=np.uint64).tobytes() + np.array([Lx, Dx, 0, 0], dtype=np.uint32).tobytes()
        hdr += np.array([labels_off, latents_off, paths_off, len(blob)], dtype=np.uint64).tobytes()
        assert len(hdr) == 64
        f.write(hdr)
    os.replace(tmp, out_path)
    return n


def write_shard(out_path: str, latents: np.ndarray, labels: np.ndarray, img_paths: Sequence[str] = ()) -> None:
    """Write an in-memory (fp32 [n, L, D], int [n]) set as a shard (same format as
    pack_latent_dir)."""
    latents = np.ascontiguousarray(latents, dtype=np.float32)
    n, Lx, Dx = latents.shape
    labels_off = 64
    latents_off = (labels_off + 4 * n + 4095) // 4096 * 4096
    paths_off = latents_off + latents.nbytes
    blob = b"\0".join(p.encode() for p in img_paths) if img_paths else b""
    hdr = MAGIC + np.array([n], dtype=np.uint64).tobytes() + np.array([Lx, Dx, 0, 0], dtype=np.uint32).tobytes()
    hdr += np.array([labels_off, latents_off, paths_off, len(blob)], dtype=np.uint64).tobytes()
    with open(out_path, "wb") as f:
        f.write(hdr)
        f.write(np.ascontiguousarray(labels, dtype=np.int32).tobytes())
        f.seek(latents_off)
        f.write(latents.tobytes())
        f.write(blob)


# ------------------------------------------------------------------ dataset
class PackedLatentDataset(torch.utils.data.Dataset):
    """LatentFERDataset over a packed shard: `ds[i] -> (latent fp32 [L, D], label)`."""

    def __init__(self, path: str, transform=None):
        L = iolib()
        h = L.fio_open(path.encode())
        if not h:
            raise RuntimeError(f"{path}: {L.fio_last_error().decode()}")
        self._h = h
        self.path = path
        self.transform = transform
        n, l_, d_ = C.c_int64(), C.c_int(), C.c_int()
        _check(L.fio_info(h, C.byref(n), C.byref(l_), C.byref(d_)), "fio_info")
        self.count, self.L, self.D = n.value, l_.value, d_.value
        self.labels = np.ctypeslib.as_array(L.fio_labels(h), shape=(self.count,)).copy()

    def __len__(self) -> int:
        return self.count

    def gather(self, idx: np.ndarray, out: torch.Tensor, labels_out: Optional[np.ndarray] = None,
               threads: int = 8) -> None:
        """out[i] = latent[idx[i]] (out: contiguous fp32 CPU tensor [len(idx), L, D])."""
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        assert out.is_contiguous() and out.dtype == torch.float32 and out.numel() >= len(idx) * self.L * self.D
        lp = None if labels_out is None else labels_out.ctypes.data
        _check(iolib().fio_gather(self._h, idx.ctypes.data, len(idx), out.data_ptr(), lp, threads), "fio_gather")

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, int]:
        if idx < 0:
            idx += self.count
        x = torch.empty(self.L, self.D, dtype=torch.float32)
        self.gather(np.array([idx]), x)
        if self.transform:
            x = self.transform(x)
        return x, int(self.labels[idx])

    def img_paths(self) -> Sequence[str]:
        blob, nb = C.c_void_p(), C.c_int64()
        _check(iolib().fio_paths(self._h, C.byref(blob), C.byref(nb)), "fio_paths")
        if nb.value == 0:
            return [""] * self.count
        return C.string_at(blob.value, nb.value).decode().split("\0")

    def get_class_counts(self) -> Dict[int, int]:
        u, c = np.unique(self.labels, return_counts=True)
        return {int(a): int(b) for a, b in zip(u, c)}

    def get_class_names(self) -> Dict[int, str]:
        return dict(CLASS_NAMES)

    def close(self) -> None:
        if getattr(self, "_h", None):
            iolib().fio_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ loader
class PackedLatentLoader:
    """Device batches (x fp32 [B, L, D], y int64 [B]) from a PackedLatentDataset.

    shuffle: a new permutation per epoch (`set_epoch`), seeded; rank / world_size split each
    epoch's order like DistributedSampler (padded to a multiple of world_size); `indices`
    restricts to a subset (e.g. the class-balanced fraction of `train_latent_vit_v2.py:42-76`).
    augment: dict(noise_std=, scale_range=(lo, hi), mask_prob=) -> LatentAugment on device.
    device=None yields pinned CPU tensors (no GPU needed)."""

    def __init__(self, dataset: PackedLatentDataset, batch_size: int, shuffle: bool = True, drop_last: bool = False,
                 seed: int = 0, device="cuda", indices: Optional[Sequence[int]] = None, rank: int = 0,
                 world_size: int = 1, threads: int = 8, augment: Optional[dict] = None):
        self.ds = dataset
        self.B = int(batch_size)
        self.shuffle, self.drop_last, self.seed = shuffle, drop_last, int(seed)
        self.device = None if device is None else torch.device(device)
        self.indices = np.arange(len(dataset), dtype=np.int64) if indices is None else np.asarray(indices, np.int64)
        self.rank, self.world = int(rank), int(world_size)
        self.threads = threads
        self.augment = augment
        self.epoch = 0
        pin = self.device is not None and self.device.type == "cuda"
        shape = (self.B, dataset.L, dataset.D)
        self._host = [torch.empty(shape, dtype=torch.float32, pin_memory=pin) for _ in range(2)]
        self._lab = [np.empty(self.B, dtype=np.int32) for _ in range(2)]
        self._ev = [None, None]

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def _order(self) -> np.ndarray:
        idx = self.indices
        if self.shuffle:
            idx = idx[np.random.default_rng(self.seed + self.epoch).permutation(len(idx))]
        if self.world > 1:
            per = -(-len(idx) // self.world)
            idx = np.concatenate([idx, idx[: per * self.world - len(idx)]])[self.rank::self.world]
        return idx

    def __len__(self) -> int:
        n = len(self._order()) if self.world > 1 else len(self.indices)
        return n // self.B if self.drop_last else -(-n // self.B)

    def __iter__(self):
        order = self._order()
        nb = len(order) // self.B if self.drop_last else -(-len(order) // self.B)
        batches = [order[k * self.B:(k + 1) * self.B] for k in range(nb)]
        ready: "queue.Queue" = queue.Queue()
        free: "queue.Queue" = queue.Queue()
        for slot in (0, 1):
            free.put(slot)
        stop = threading.Event()

        def producer():
            # gathers batch k+1 into the other pinned buffer while batch k is consumed; a buffer is
            # reused only after the consumer handed it back (copy enqueued) and that copy finished
            try:
                for k, bi in enumerate(batches):
                    slot = free.get()
                    if stop.is_set():
                        return
                    ev = self._ev[slot]
                    if ev is not None:
                        ev.synchronize()
                    self.ds.gather(bi, self._host[slot], self._lab[slot], self.threads)
                    ready.put((k, slot, len(bi)))
                ready.put(None)
            except BaseException as e:  # surface reader errors in the consumer
                ready.put(e)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        side = torch.cuda.Stream(self.device) if self.device is not None and self.device.type == "cuda" else None
        try:
            while True:
                item = ready.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                k, slot, n = item
                xh = self._host[slot][:n]
                yh = torch.from_numpy(self._lab[slot][:n].astype(np.int64))
                if side is None:
                    x = xh.clone()
                    free.put(slot)
                    yield x, yh
                    continue
                with torch.cuda.stream(side):
                    x = xh.to(self.device, non_blocking=True)
                    y = yh.to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(side)
                self._ev[slot] = ev
                free.put(slot)
                cur = torch.cuda.current_stream(self.device)
                cur.wait_stream(side)
                x.record_stream(cur)
                y.record_stream(cur)
                if self.augment:
                    self._augment(x, k)
                yield x, y
        finally:
            stop.set()
            free.put(0)  # unblock a producer waiting for a slot
            th.join()
            self.epoch += 1

    def _augment(self, x: torch.Tensor, k: int) -> None:
        from . import ops
        from ._lib import check, lib

        a = self.augment
        lo, hi = a.get("scale_range") or (1.0, 1.0)
        seed = (self.seed * 0x9E3779B97F4A7C15 + (self.epoch << 32) + k * 0xBF58476D1CE4E5B9 + self.rank) % (1 << 64)
        check(lib().fer_latent_augment(x.data_ptr(), x.shape[0], x.shape[1] * x.shape[2], float(a.get("noise_std", 0.0)),
                                       float(lo), float(hi), float(a.get("mask_prob", 0.0)), seed, ops.stream()),
              "latent_augment")
