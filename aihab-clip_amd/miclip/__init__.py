"""miclip: MI355X-native CLIP encode path behind the reference `clip` API.

    import miclip as clip
    state_dict, model, preprocess = clip.load("ViT-L/14", device="cuda")
    feats = model.encode_image(images)            # [B, 1024] pre-projection
    x_before, x = model.encode_text(tokens)       # tuple, like clip/model.py:338-353

Everything on the encode path runs in hand-written CDNA4 HIP kernels behind the
C ABI of libmiclip.so (include/miclip.h); there is no CPU fallback.
"""
import os
import warnings

import torch

from .configs import (MODEL_CONFIGS, OPEN_CLIP_MODELS, CLIPConfig, available_models,
                      config_from_state_dict)
from .model import CLIP, build_model
from .preprocess import Transform
from .weights import generate_state_dict, synthetic_images

__all__ = ["available_models", "load", "tokenize", "build_model", "CLIP", "CLIPConfig",
           "MODEL_CONFIGS", "SeededWeightsWarning"]


class SeededWeightsWarning(UserWarning):
    """A model name (or, with allow_seeded=True, an open_clip pretrained tag) was
    resolved to seeded random weights: no checkpoints exist offline. Filter it where
    that is intended (benchmarks, tests); pass a state-dict path for real weights."""


def _transform(n_px):
    return Transform(n_px)


def load(name, device="cuda" if torch.cuda.is_available() else "cpu", jit=False,
         download_root=None, *, seed: int = 0, compute_dtype: str = "fp16", surface=None,
         config=None, options=None):
    """Counterpart of clip.load (clip/clip.py:89-137): returns (state_dict, model, preprocess).

    `name` is a model name from available_models() -- resolved offline to the
    CLIP shapes with seeded random weights (no checkpoints exist offline; a
    SeededWeightsWarning says so) -- or
    a path to a state-dict checkpoint (loaded with weights_only=True). Anything
    else raises RuntimeError like the reference. `jit=True` is accepted with a
    warning and loads the non-JIT model (the reference does the same when the
    file is not a JIT archive, clip/clip.py:127-130). `download_root` is unused.
    `surface` picks the model's call contract: "openai" (the vendored
    clip/model.py: pre-projection encode_image, tuple encode_text) or
    "open_clip" (post-projection, one tensor; methods/PEFT_openclip.py); it
    defaults to "open_clip" for open_clip model names (OPEN_CLIP_MODELS).
    `config` (a CLIPConfig or a MODEL_CONFIGS name) fixes the architecture of a
    state-dict file instead of inferring it: shape inference (build_model) cannot
    see the activation or the vision head width, so an open_clip ViT-H-14 file
    needs config="ViT-H-14" (exact GELU, 16 heads of 80); every tensor's shape is
    then checked against that config. `options` ({name: bool}, model.OPTIONS)
    selects a non-default numerics path (e.g. {"resid_f32": True}); the library
    reads no environment variables.
    """
    if surface is None:
        surface = "open_clip" if name in OPEN_CLIP_MODELS else "openai"
    if name in MODEL_CONFIGS:
        warnings.warn(f"{name}: no checkpoint offline; loading SEEDED RANDOM weights (seed={seed}). "
                      f"Pass a state-dict file path for real weights.", SeededWeightsWarning,
                      stacklevel=2)
        cfg = MODEL_CONFIGS[name]
        sd = generate_state_dict(cfg, seed=seed)
        sd = {k: torch.from_numpy(v) for k, v in sd.items()}
    elif os.path.isfile(name):
        sd = torch.load(name, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd and "visual.proj" not in sd:
            sd = sd["state_dict"]
        for key in ("input_resolution", "context_length", "vocab_size"):
            sd.pop(key, None)
        cfg = config_from_state_dict(sd)
        if config is not None:
            cfg = _checked_config(config, sd, name)
    else:
        raise RuntimeError(f"Model {name} not found; available models = {available_models()}")
    if jit:
        warnings.warn(f"{name}: JIT archives are not supported by miclip; loading as a state dict")
    model = CLIP(cfg, sd, device=device, compute_dtype=compute_dtype, surface=surface,
                 options=options).eval()
    return model.state_dict(), model, _transform(cfg.image_resolution)


def _checked_config(config, sd, name):
    from .weights import param_specs
    cfg = MODEL_CONFIGS[config] if isinstance(config, str) else config
    for key, shape, _, _ in param_specs(cfg):
        if key not in sd:
            raise RuntimeError(f"{name}: missing key {key!r} for the given config")
        if tuple(sd[key].shape) != tuple(shape):
            raise RuntimeError(f"{name}: {key} has shape {tuple(sd[key].shape)}, the config "
                               f"expects {tuple(shape)}")
    return cfg


def tokenize(texts, context_length: int = 77, truncate: bool = False):
    from .tokenizer import tokenize as _tokenize
    return _tokenize(texts, context_length, truncate)
