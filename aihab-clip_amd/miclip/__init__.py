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
           "MODEL_CONFIGS"]


def _transform(n_px):
    return Transform(n_px)


def load(name, device="cuda" if torch.cuda.is_available() else "cpu", jit=False,
         download_root=None, *, seed: int = 0, compute_dtype: str = "fp16", surface=None):
    """Counterpart of clip.load (clip/clip.py:89-137): returns (state_dict, model, preprocess).

    `name` is a model name from available_models() -- resolved offline to the
    CLIP shapes with seeded random weights (no checkpoints exist offline) -- or
    a path to a state-dict checkpoint (loaded with weights_only=True). Anything
    else raises RuntimeError like the reference. `jit=True` is accepted with a
    warning and loads the non-JIT model (the reference does the same when the
    file is not a JIT archive, clip/clip.py:127-130). `download_root` is unused.
    `surface` picks the model's call contract: "openai" (the vendored
    clip/model.py: pre-projection encode_image, tuple encode_text) or
    "open_clip" (post-projection, one tensor; methods/PEFT_openclip.py); it
    defaults to "open_clip" for open_clip model names (OPEN_CLIP_MODELS).
    """
    if surface is None:
        surface = "open_clip" if name in OPEN_CLIP_MODELS else "openai"
    if name in MODEL_CONFIGS:
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
    else:
        raise RuntimeError(f"Model {name} not found; available models = {available_models()}")
    if jit:
        warnings.warn(f"{name}: JIT archives are not supported by miclip; loading as a state dict")
    model = CLIP(cfg, sd, device=device, compute_dtype=compute_dtype, surface=surface).eval()
    return model.state_dict(), model, _transform(cfg.image_resolution)


def tokenize(texts, context_length: int = 77, truncate: bool = False):
    from .tokenizer import tokenize as _tokenize
    return _tokenize(texts, context_length, truncate)
