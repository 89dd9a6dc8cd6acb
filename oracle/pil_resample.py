"""CPU oracle: restatement of the reference's CLIP image preprocessing.

TEST INFRASTRUCTURE ONLY (same import rule as clip_oracle.py: tests/, smoke()
and bench.py's cpu_baseline leg only).

The reference preprocesses every image on the CPU with torchvision on a PIL
image:
  * `_transform(n_px)`               clip/clip.py:74-81
  * `build_clip_transforms(…, False)` data/clip_transforms.py:50-55 (test split)
both = Resize(n_px, BICUBIC) on the shorter side -> CenterCrop(n_px) -> RGB ->
ToTensor -> Normalize(CLIP_MEAN, CLIP_STD) (data/clip_transforms.py:22-23).

The arithmetic lives in two third-party packages that are not vendored in the
reference:
  * torchvision (absent from this image, version unpinned by the reference):
    output size `_compute_resized_output_size` (short side -> n_px, long side
    -> int(n_px * long / short)), center-crop anchor int(round((h - n)/2.0))
    (Python round: half to even), ToTensor = uint8 -> float32 / 255,
    Normalize = (x - mean) / std in float32.
  * Pillow (present in this image, 12.2.0): `Image.resize(size, BICUBIC)` ->
    libImaging/Resample.c: `precompute_coeffs` (double coefficients of the
    a = -0.5 cubic, support 2 * max(scale, 1), normalised per output pixel),
    `normalize_coeffs_8bpc` (fixed point, PRECISION_BITS = 22, round half away
    from zero), horizontal pass then vertical pass over 8-bit data, each
    output = clip8((1 << 21) + sum(u8 * coeff)) with clip8(v) = clamp(v >> 22, 0, 255).

`resize_bicubic_u8` restates Resample.c in numpy with the same double
operation order; tests/test_preprocess.py pins it against Pillow itself
(bit-exact uint8), and `transform_reference` (Pillow's own resize + the
torchvision steps above) is the checker of the HIP preprocessing kernel.
"""
import math

import numpy as np

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)
PRECISION_BITS = 32 - 8 - 2


def output_size(h, w, n_px):
    """torchvision `_compute_resized_output_size` for an int size: (new_h, new_w)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = n_px, int(n_px * long / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def crop_anchor(h, w, n_px):
    """torchvision center-crop anchor (top, left) = int(round((size - n)/2.0))."""
    return int(round((h - n_px) / 2.0)), int(round((w - n_px) / 2.0))


def _bicubic(x):
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs(in_size, out_size):
    """Resample.c precompute_coeffs + normalize_coeffs_8bpc (box = whole input).

    Returns (bounds [out, 2] int: xmin, count; kk [out, ksize] int64 fixed point).
    """
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        k = [0.0] * xmax
        for x in range(xmax):
            w = _bicubic((x + xmin - center + 0.5) * ss)
            k[x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                k[x] /= ww
        for x in range(xmax):
            v = k[x] * (1 << PRECISION_BITS)
            kk[xx, x] = int(-0.5 + v) if k[x] < 0 else int(0.5 + v)
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(src, bounds, kk, axis):
    """One 8-bit resampling pass along `axis` (0 = rows/vertical, 1 = columns)."""
    src = np.moveaxis(src.astype(np.int64), axis, 0)
    out = np.empty((bounds.shape[0],) + src.shape[1:], np.uint8)
    for o in range(bounds.shape[0]):
        xmin, n = bounds[o]
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += src[xmin + t] * kk[o, t]
        out[o] = np.clip(acc >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis)


def resize_bicubic_u8(img, size):
    """Pillow Image.resize((w, h), BICUBIC) on an HxWxC uint8 array; size = (h, w)."""
    h, w = img.shape[:2]
    oh, ow = size
    x = img
    if ow != w:
        b, k = precompute_coeffs(w, ow)
        x = _pass(x, b, k, 1)
    if oh != h:
        b, k = precompute_coeffs(h, oh)
        x = _pass(x, b, k, 0)
    return x


def to_rgb(img):
    """HxW or HxWx{1,3} uint8 -> HxWx3 (PIL convert('RGB') of an 'L' image replicates)."""
    if img.ndim == 2:
        img = img[:, :, None]
    if img.shape[2] == 1:
        img = np.repeat(img, 3, axis=2)
    return img


def crop_u8(img, n_px, resize=resize_bicubic_u8):
    """Resize (shorter side -> n_px) + center crop of an HxWxC uint8 image."""
    h, w = img.shape[:2]
    nh, nw = output_size(h, w, n_px)
    r = resize(img, (nh, nw))
    top, left = crop_anchor(nh, nw, n_px)
    return r[top:top + n_px, left:left + n_px]


def normalize(u8):
    """ToTensor + Normalize of an n x n x 3 uint8 crop -> float32 [3, n, n]."""
    a = u8.astype(np.float32) / np.float32(255.0)
    a = (a - np.asarray(CLIP_MEAN, np.float32)) / np.asarray(CLIP_STD, np.float32)
    return np.ascontiguousarray(a.transpose(2, 0, 1))


def pil_resize(img, size):
    """Pillow itself (the third-party implementation the reference calls)."""
    from PIL import Image
    mode = "L" if img.ndim == 2 or img.shape[2] == 1 else "RGB"
    im = Image.fromarray(img.reshape(img.shape[0], img.shape[1]) if mode == "L" else img, mode)
    out = np.asarray(im.resize((size[1], size[0]), Image.BICUBIC))
    return out if out.ndim == 3 else out[:, :, None]


def transform_reference(img, n_px):
    """Reference preprocessing of one uint8 image with Pillow's resize -> float32 [3,n,n]."""
    return normalize(to_rgb(crop_u8(img, n_px, resize=pil_resize)))
