"""Deterministic, counter-based weight and input generator.

There are no CLIP checkpoints offline, so every model name
resolves to seeded random weights with the exact CLIP state-dict keys and
shapes (clip/model.py:238-329; key order as `CLIP.state_dict()`).

Each tensor is drawn from its own Philox stream keyed by (seed, crc32(name)),
so the GPU box regenerates bit-identical weights without shipping any file,
and a tensor does not change when another one is added or resized.

Init stds follow the reference's `initialize_parameters` /
`VisionTransformer.__init__` (clip/model.py:206-214, 294-321), applied to the
visual blocks too; biases and LayerNorm affine params are drawn non-trivially
(the reference leaves them 0/1) so that every bias / LN epilogue of the HIP
path is exercised by the parity tests.
"""
import zlib
from collections import OrderedDict

import numpy as np

from .configs import CLIPConfig

# clip/clip.py:80 (Normalize(...)), also data/clip_transforms.py:22-23
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.Philox(key=[int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                     zlib.crc32(name.encode())]))


def _normal(seed, name, shape, std, mean=0.0):
    a = _rng(seed, name).standard_normal(int(np.prod(shape)) if shape else 1, dtype=np.float32)
    a = a.reshape(shape) * np.float32(std)
    if mean:
        a = a + np.float32(mean)
    return a.astype(np.float32, copy=False)


def _block_specs(prefix, width, layers):
    proj_std = (width ** -0.5) * ((2 * layers) ** -0.5)     # clip/model.py:311
    attn_std = width ** -0.5                                # clip/model.py:312
    fc_std = (2 * width) ** -0.5                            # clip/model.py:313
    out = []
    for i in range(layers):
        p = f"{prefix}resblocks.{i}."
        out += [
            (p + "attn.in_proj_weight", (3 * width, width), attn_std, 0.0),
            (p + "attn.in_proj_bias", (3 * width,), 0.02, 0.0),
            (p + "attn.out_proj.weight", (width, width), proj_std, 0.0),
            (p + "attn.out_proj.bias", (width,), 0.02, 0.0),
            (p + "ln_1.weight", (width,), 0.1, 1.0),
            (p + "ln_1.bias", (width,), 0.05, 0.0),
            (p + "mlp.c_fc.weight", (4 * width, width), fc_std, 0.0),
            (p + "mlp.c_fc.bias", (4 * width,), 0.02, 0.0),
            (p + "mlp.c_proj.weight", (width, 4 * width), proj_std, 0.0),
            (p + "mlp.c_proj.bias", (width,), 0.02, 0.0),
            (p + "ln_2.weight", (width,), 0.1, 1.0),
            (p + "ln_2.bias", (width,), 0.05, 0.0),
        ]
    return out


def param_specs(cfg: CLIPConfig):
    """(name, shape, std, mean) for every state-dict tensor, in CLIP.state_dict() order."""
    Wv, Wt, E, P = cfg.vision_width, cfg.transformer_width, cfg.embed_dim, cfg.vision_patch_size
    vscale = Wv ** -0.5                                     # clip/model.py:206
    specs = [
        ("positional_embedding", (cfg.context_length, Wt), 0.01, 0.0),     # :296
        ("text_projection", (Wt, E), Wt ** -0.5, 0.0),                     # :321
        ("logit_scale", (), 0.0, float(np.log(1 / 0.07))),                # :290
        ("visual.class_embedding", (Wv,), vscale, 0.0),                   # :207
        ("visual.positional_embedding", (cfg.n_tokens, Wv), vscale, 0.0),  # :208
        ("visual.proj", (Wv, E), vscale, 0.0),                            # :214
        ("visual.conv1.weight", (Wv, 3, P, P), (3 * P * P) ** -0.5, 0.0),
        ("visual.ln_pre.weight", (Wv,), 0.1, 1.0),
        ("visual.ln_pre.bias", (Wv,), 0.05, 0.0),
    ]
    specs += _block_specs("visual.transformer.", Wv, cfg.vision_layers)
    specs += [
        ("visual.ln_post.weight", (Wv,), 0.1, 1.0),
        ("visual.ln_post.bias", (Wv,), 0.05, 0.0),
    ]
    specs += _block_specs("transformer.", Wt, cfg.transformer_layers)
    specs += [
        ("token_embedding.weight", (cfg.vocab_size, Wt), 0.02, 0.0),      # :295
        ("ln_final.weight", (Wt,), 0.1, 1.0),
        ("ln_final.bias", (Wt,), 0.05, 0.0),
    ]
    return specs


def _fp16_stored(name: str) -> bool:
    """Tensors the reference keeps in fp16 (convert_weights, clip/model.py:372-393):
    Conv/Linear weight+bias, MHA in_proj_weight/in_proj_bias, `proj`, `text_projection`.
    clip.load round-trips them through fp16 even on CPU (build_model casts, then
    clip/clip.py:135-136 calls .float()), so the generator draws them fp16-exact."""
    if name in ("visual.proj", "text_projection", "visual.conv1.weight"):
        return True
    return (".attn." in name or ".mlp." in name) and not name.endswith("ln")


def generate_state_dict(cfg: CLIPConfig, seed: int = 0, towers=("visual", "text")):
    """OrderedDict name -> float32 numpy array. `towers` can skip a tower's big tensors."""
    sd = OrderedDict()
    for name, shape, std, mean in param_specs(cfg):
        is_visual = name.startswith("visual.")
        if is_visual and "visual" not in towers:
            continue
        if not is_visual and name not in ("logit_scale",) and "text" not in towers:
            continue
        if std == 0.0:
            sd[name] = np.full(shape, mean, dtype=np.float32)
        else:
            a = _normal(seed, name, shape, std, mean)
            if _fp16_stored(name):
                a = a.astype(np.float16).astype(np.float32)
            sd[name] = a
    return sd


def _halton(i: int, base: int) -> float:
    f, r = 1.0, 0.0
    while i > 0:
        f /= base
        r += f * (i % base)
        i //= base
    return r


def _bilinear_grid(g: np.ndarray, R: int) -> np.ndarray:
    """[C, k, k] control grid -> [C, R, R] by bilinear interpolation at pixel centres."""
    k = g.shape[1]
    t = (np.arange(R, dtype=np.float64) + 0.5) / R * (k - 1)
    i0 = np.clip(np.floor(t).astype(np.int64), 0, k - 2)
    f = t - i0
    rows = g[:, i0, :] * (1 - f)[None, :, None] + g[:, i0 + 1, :] * f[None, :, None]
    return rows[:, :, i0] * (1 - f)[None, None, :] + rows[:, :, i0 + 1] * f[None, None, :]


def _structured_image(seed: int, resolution: int, j: int) -> np.ndarray:
    """Image j of the structured set, pixel values in [0, 1], [3, R, R] float32.

    A low-frequency random field (bilinear over a k x k grid, k in 2..8) plus three
    oriented gratings, scaled by a per-channel contrast (log-uniform 0.05..0.5) around
    a per-image base colour taken from a Halton sequence (so the base colours of any
    16 consecutive images are well spread), plus a little pixel noise, clipped to
    [0, 1]. Unlike i.i.d. noise, whose CLIP embeddings share ~95 % of their norm,
    these give image-specific features (inter-image 1-cos >= 1.6e-2 over the
    fixtures' 16 images on random-init ViT-B/32 and ViT-L/14)."""
    R = resolution
    r = _rng(seed, f"structured/{R}/{j}")
    k = int(r.integers(2, 9))
    img = _bilinear_grid(r.standard_normal((3, k, k)), R)
    c = (np.arange(R, dtype=np.float64) + 0.5) / R
    for _ in range(3):
        fx, fy = r.uniform(-12, 12, 2)
        ph = r.uniform(0, 2 * np.pi)
        amp = r.uniform(0, 0.6, 3)
        wave = np.sin(2 * np.pi * (fy * c[:, None] + fx * c[None, :]) + ph)
        img += amp[:, None, None] * wave[None]
    contrast = np.exp(r.uniform(np.log(0.05), np.log(0.5), 3))
    base = 0.1 + 0.8 * np.array([_halton(j + 1, 2), _halton(j + 1, 3), _halton(j + 1, 5)])
    img = base[:, None, None] + contrast[:, None, None] * img
    img += 0.02 * r.standard_normal(img.shape)
    return np.clip(img, 0.0, 1.0).astype(np.float32)


def synthetic_images(batch: int, resolution: int, seed: int = 0, offset: int = 0,
                     kind: str = "structured") -> np.ndarray:
    """CLIP-normalised synthetic images [B,3,R,R] float32: (u - mean_c) / std_c.

    Same normalisation as the reference preprocess (clip/clip.py:80). Image i of
    the set is drawn from its own stream, so a shard [offset, offset+batch)
    equals the same rows of a full batch. kind="structured" (default since r04):
    per-image low-frequency fields, gratings, base colour and contrast
    (`_structured_image`), so embeddings of different images differ well beyond
    the parity tolerance; kind="noise": u ~ U[0,1) per pixel (the r01-r03 fixtures).
    """
    out = np.empty((batch, 3, resolution, resolution), dtype=np.float32)
    mean = np.asarray(CLIP_MEAN, np.float32)[:, None, None]
    std = np.asarray(CLIP_STD, np.float32)[:, None, None]
    for i in range(batch):
        if kind == "structured":
            u = _structured_image(seed, resolution, offset + i)
        elif kind == "noise":
            u = _rng(seed, f"image/{resolution}/{offset + i}").random(
                (3, resolution, resolution), dtype=np.float32)
        else:
            raise ValueError(f"unknown synthetic image kind {kind!r}")
        out[i] = (u - mean) / std
    return out


def checksum(a: np.ndarray) -> str:
    """crc32 of the raw bytes; used by fixtures to detect generator drift."""
    return format(zlib.crc32(np.ascontiguousarray(a).tobytes()), "08x")
