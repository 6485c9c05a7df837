"""CPU oracle for the ImageViT input transforms (TEST INFRASTRUCTURE ONLY: imported by tests/
and tests/golden/make_image_golden.py as the checker, never by the product path).

The reference runs torchvision transforms on PIL images, `data/image_dataset.py:139-173`
(get_train_transforms / get_val_transforms; images opened with `.convert('RGB')`,
`data/image_dataset.py:126`). Pillow is installed here (12.2; reference pins Pillow>=8.0) and
every pixel operation below IS Pillow's. torchvision (reference pins >=0.15) is not installed,
so its thin glue between the Pillow calls is restated from its published functional API:
  * RandomHorizontalFlip -> img.transpose(FLIP_LEFT_RIGHT)
  * RandomRotation(15)   -> img.rotate(angle, NEAREST, expand=False, fillcolor=0)
                            (transforms.functional.rotate -> functional_pil.rotate)
  * ColorJitter          -> ImageEnhance.Brightness / Contrast / Color .enhance(f) in the
                            randperm order; adjust_hue = HSV split, h += uint8(hf*255), merge
  * RandomAffine         -> img.transform(size, AFFINE, _get_inverse_affine_matrix(center=
                            (w*0.5, h*0.5), angle=0, (tx, ty), scale, shear=0), NEAREST, fill 0)
  * ToTensor/Normalize   -> uint8 / 255 then (x - mean) / std in fp32
Random draws are explicit (the parameter record the kernel consumes), so a test feeds the
same parameters to both sides. Parity target: bit-exact uint8 stages, hence outputs equal to
fp32 rounding of the same division.
"""
from __future__ import annotations

import math

import numpy as np
from PIL import Image, ImageEnhance

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)

# parameter record layout (include/fervit.h fer_image_augment)
P_FLIP, P_ANGLE, P_BRIGHT, P_CONTRAST, P_SAT, P_HUE, P_ORDER, P_TX, P_TY, P_SCALE, P_HUE_ON = 0, 1, 2, 3, 4, 5, 6, 10, 11, 12, 13


def adjust_hue(img: Image.Image, hue_factor: float) -> Image.Image:
    """torchvision functional_pil.adjust_hue."""
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    np_h += np.array(hue_factor * 255).astype(np.uint8)  # wraps, as torchvision intends
    h = Image.fromarray(np_h, "L")
    return Image.merge("HSV", (h, s, v)).convert("RGB")


def affine_matrix(S: int, tx: int, ty: int, scale: float) -> list:
    """torchvision _get_inverse_affine_matrix for angle 0 / shear 0 (the RandomAffine of the
    reference), PIL branch center = (w*0.5, h*0.5)."""
    cx, cy = S * 0.5, S * 0.5
    rot, sx, sy = 0.0, 0.0, 0.0
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m = [x / scale for x in m]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def val_uint8(img: Image.Image, S: int) -> np.ndarray:
    """Resize((S,S)) of an RGB image -> uint8 [S][S][3]."""
    return np.asarray(img.convert("RGB").resize((S, S), Image.BILINEAR))


def train_uint8(img: Image.Image, S: int, p) -> np.ndarray:
    """get_train_transforms up to ToTensor, with the parameter record p -> uint8 [S][S][3]."""
    im = img.convert("RGB").resize((S, S), Image.BILINEAR)
    if p[P_FLIP]:
        im = im.transpose(Image.FLIP_LEFT_RIGHT)
    im = im.rotate(float(p[P_ANGLE]), Image.NEAREST, expand=False, fillcolor=(0, 0, 0))
    for op in [int(v) for v in p[P_ORDER:P_ORDER + 4]]:
        f = float(p[P_BRIGHT + op])
        if op == 0:
            im = ImageEnhance.Brightness(im).enhance(f)
        elif op == 1:
            im = ImageEnhance.Contrast(im).enhance(f)
        elif op == 2:
            im = ImageEnhance.Color(im).enhance(f)
        elif p[P_HUE_ON]:  # ColorJitter(hue=0) has hue None and skips the HSV round trip
            im = adjust_hue(im, f)
    m = affine_matrix(S, int(p[P_TX]), int(p[P_TY]), float(p[P_SCALE]))
    im = im.transform((S, S), Image.AFFINE, m, Image.NEAREST, fillcolor=(0, 0, 0))
    return np.asarray(im)


def normalize(u8: np.ndarray) -> np.ndarray:
    """ToTensor + Normalize: uint8 HWC -> fp32 CHW."""
    x = u8.astype(np.float32).transpose(2, 0, 1) / np.float32(255.0)
    return (x - MEAN[:, None, None]) / STD[:, None, None]


def random_params(n: int, S: int, rng: np.random.Generator, degrees=15.0, b=0.2, c=0.2, s=0.2, h=0.1,
                  translate=0.1, scale=(0.9, 1.1)) -> np.ndarray:
    """Parameter records drawn like torchvision's get_params (fp32 draws, as torch's are)."""
    P = np.zeros((n, 16), dtype=np.float32)
    for i in range(n):
        P[i, P_FLIP] = float(rng.random() < 0.5)
        P[i, P_ANGLE] = rng.uniform(-degrees, degrees)
        P[i, P_BRIGHT] = rng.uniform(max(0, 1 - b), 1 + b)
        P[i, P_CONTRAST] = rng.uniform(max(0, 1 - c), 1 + c)
        P[i, P_SAT] = rng.uniform(max(0, 1 - s), 1 + s)
        P[i, P_HUE] = rng.uniform(-h, h)
        P[i, P_ORDER:P_ORDER + 4] = rng.permutation(4)
        md = translate * S
        P[i, P_TX] = int(round(float(np.float32(rng.uniform(-md, md)))))
        P[i, P_TY] = int(round(float(np.float32(rng.uniform(-md, md)))))
        P[i, P_SCALE] = rng.uniform(*scale)
        P[i, P_HUE_ON] = float(h > 0)
    return P
