"""ImageViT input transforms on the GPU.

Drop-in for `data/image_dataset.py:139-173`: `get_train_transforms(img_size)` /
`get_val_transforms(img_size)` return batch transforms that take the decoded images of a batch
(PIL images or uint8 HWC arrays, any size, grey or RGB) and return the normalised fp32 NCHW
device batch the ImageViT patch embedding consumes. The per-image torchvision chain (Resize,
flip, rotation, ColorJitter, affine, ToTensor, Normalize) runs as one HIP kernel per batch
(`fer_image_augment`, csrc/image.hip) that follows Pillow's arithmetic, so for the same random
parameters the pixels equal the reference's; parameters are drawn on device
(`fer_image_aug_draw`) from a counter hash with torchvision's ranges.

Decoding stays on the host (the reference's `Image.open(...).convert('RGB')`,
`data/image_dataset.py:126`); the sources travel to HBM packed in one pinned buffer.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np
import torch

from . import ops
from ._lib import ImageAug, check, lib
from .runtime import next_seed

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _as_hwc(img) -> np.ndarray:
    mode = getattr(img, "mode", None)
    if mode is not None and mode not in ("L", "RGB"):
        img = img.convert("RGB")  # palette / CMYK / ... as the reference's convert('RGB')
    a = np.asarray(img)
    if a.dtype != np.uint8:
        raise TypeError("images must be uint8 (decoded PIL images or HWC arrays)")
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim != 3 or a.shape[2] not in (1, 3, 4):
        raise ValueError(f"image shape {a.shape} is not HW, HWC with C in (1, 3) or RGBA")
    if a.shape[2] == 4:  # convert('RGB') drops alpha
        a = a[:, :, :3]
    return np.ascontiguousarray(a)


class GPUImageTransform:
    """Batched transform: `t(images, params=None) -> fp32 [B, 3, S, S]` on the current device.

    train=False is get_val_transforms; train=True is get_train_transforms with the reference's
    ranges (overridable). `params` (fp32 [B, 16] device tensor, layout in include/fervit.h)
    replaces the device draw, e.g. to replay a batch; `last_params` keeps the last records."""

    def __init__(self, img_size: int = 224, train: bool = True, flip_p: float = 0.5, degrees: float = 15.0,
                 brightness: float = 0.2, contrast: float = 0.2, saturation: float = 0.2, hue: float = 0.1,
                 translate: float = 0.1, scale=(0.9, 1.1), mean=IMAGENET_MEAN, std=IMAGENET_STD):
        if not 0 < img_size <= 1024:
            raise ValueError("img_size must be in (0, 1024]")
        self.img_size = int(img_size)
        self.train = bool(train)
        self.aug = ImageAug(flip_p, degrees, brightness, contrast, saturation, hue, translate, scale[0], scale[1])
        self.mean = (C.c_float * 3)(*mean)
        self.std = (C.c_float * 3)(*std)
        self.last_params: Optional[torch.Tensor] = None

    def pack(self, images: Sequence, device=None):
        """uint8 sources -> (device bytes, offsets int64 [B], hwc int32 [B*3]) via one pinned H2D copy."""
        arrs = [_as_hwc(im) for im in images]
        sizes = [a.nbytes for a in arrs]
        offs = np.zeros(len(arrs), dtype=np.int64)
        if arrs:
            offs[1:] = np.cumsum(sizes)[:-1]
        total = int(sum(sizes))
        host = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        hv = host.numpy()
        for a, o in zip(arrs, offs):
            hv[o:o + a.nbytes] = a.reshape(-1)
        hwc = np.array([s for a in arrs for s in a.shape], dtype=np.int32)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        pin = torch.cuda.is_available()
        offs_t, hwc_t = torch.from_numpy(offs), torch.from_numpy(hwc)
        if pin:
            offs_t, hwc_t = offs_t.pin_memory(), hwc_t.pin_memory()
        return (host.to(dev, non_blocking=True), offs_t.to(dev, non_blocking=True), hwc_t.to(dev, non_blocking=True))

    def __call__(self, images: Sequence, params: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, S = len(images), self.img_size
        src, offs, hwc = self.pack(images)
        out = torch.empty(B, 3, S, S, device=src.device, dtype=torch.float32)
        if B == 0:
            return out
        prm = None
        if self.train:
            if params is None:
                prm = torch.empty(B, 16, device=src.device, dtype=torch.float32)
                check(lib().fer_image_aug_draw(prm.data_ptr(), B, S, C.byref(self.aug), next_seed(), ops.stream()),
                      "image_aug_draw")
            else:
                prm = params.to(device=src.device, dtype=torch.float32).contiguous()
                if tuple(prm.shape) != (B, 16):
                    raise ValueError("params must be [B, 16]")
            self.last_params = prm
        check(lib().fer_image_augment(src.data_ptr(), offs.data_ptr(), hwc.data_ptr(), B, S,
                                      prm.data_ptr() if prm is not None else None, int(self.train), self.mean,
                                      self.std, out.data_ptr(), ops.stream()), "image_augment")
        return out


def get_train_transforms(img_size: int = 224) -> GPUImageTransform:
    """`data/image_dataset.py:139-161` as a device batch transform."""
    return GPUImageTransform(img_size, train=True)


def get_val_transforms(img_size: int = 224) -> GPUImageTransform:
    """`data/image_dataset.py:164-173` as a device batch transform."""
    return GPUImageTransform(img_size, train=False)
