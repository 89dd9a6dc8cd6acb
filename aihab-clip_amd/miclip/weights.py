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


def synthetic_images(batch: int, resolution: int, seed: int = 0, offset: int = 0) -> np.ndarray:
    """CLIP-normalised synthetic images [B,3,R,R] float32: (U[0,1) - mean_c) / std_c.

    Same normalisation as the reference preprocess (clip/clip.py:80). Image i of
    the set is drawn from its own stream, so a shard [offset, offset+batch)
    equals the same rows of a full batch.
    """
    out = np.empty((batch, 3, resolution, resolution), dtype=np.float32)
    mean = np.asarray(CLIP_MEAN, np.float32)[:, None, None]
    std = np.asarray(CLIP_STD, np.float32)[:, None, None]
    for i in range(batch):
        u = _rng(seed, f"image/{resolution}/{offset + i}").random(
            (3, resolution, resolution), dtype=np.float32)
        out[i] = (u - mean) / std
    return out


def checksum(a: np.ndarray) -> str:
    """crc32 of the raw bytes; used by fixtures to detect generator drift."""
    return format(zlib.crc32(np.ascontiguousarray(a).tobytes()), "08x")
