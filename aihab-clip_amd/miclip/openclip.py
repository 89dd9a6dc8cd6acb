"""open_clip entry points the reference's open_clip path calls, on the HIP model.

aihab_utils/model_init.py:42-112 loads the PEFT_openclip backbone with
`open_clip.create_model_and_transforms(backbone, pretrained=..., device=...)`
and tokenises with `open_clip.get_tokenizer(backbone)`; methods/PEFT_openclip.py
then calls `model.encode_image(images)` (post-projection, :90-92) and
`model.encode_text(tokens)` (one tensor, :38-47). open_clip itself is not in
this image and the reference pins no version of it, so what is restated here is
the contract those call sites use, on miclip's open_clip surface
(`CLIP(surface="open_clip")`, model.py) -- parity unpinned with respect to
open_clip's own code.

  * create_model_and_transforms -> (model, preprocess_train, preprocess_val):
    `pretrained` = a state-dict file (built with the named model's config: exact
    GELU and 80-wide vision heads for ViT-H-14, shapes checked), or None /
    "seeded" for seeded weights of the named shape. A pretrained TAG (e.g.
    "openai", the reference config's default, or "laion2b_s32b_b79k") has no
    checkpoint offline: it loads the seeded weights with a SeededWeightsWarning,
    the same policy as `miclip.load(<model name>)`, so the reference's configs run
    unchanged and random weights are never silent.
    Both transforms are the eval transform (Resize
    bicubic + CenterCrop + CLIP normalise, open_clip's default for the OpenAI
    mean/std): the training-time augmentation is outside the encode path.
  * get_tokenizer(name) -> callable(texts, context_length=77): the CLIP BPE
    (open_clip's SimpleTokenizer is the same vocabulary and padding).

Scope: the inference contract only -- model_init, feature caching and eval.
The PEFT training loop (methods/PEFT_openclip.py:197-273: lock_image_tower /
lock_text_tower, backward through encode_image) is outside the encode path; the
model's lock_* methods raise NotImplementedError saying so.
"""
import os
import warnings

import torch

from .configs import OPEN_CLIP_MODELS


def list_models():
    return sorted(OPEN_CLIP_MODELS)


def create_model(model_name, pretrained=None, device="cuda", *, compute_dtype="fp16", seed=0,
                 allow_seeded=False, **_unused):
    from . import SeededWeightsWarning, load
    from .configs import MODEL_CONFIGS
    if model_name not in OPEN_CLIP_MODELS:
        raise RuntimeError(f"Model config for {model_name} not found; available models "
                           f"{list_models()}.")
    if pretrained not in (None, "", "seeded") and os.path.isfile(str(pretrained)):
        # the named model's architecture, not build_model's shape inference (which
        # would give QuickGELU and 64-wide heads); load() checks every shape
        src, config = str(pretrained), MODEL_CONFIGS[model_name]
    else:
        if pretrained not in (None, "", "seeded"):
            # a checkpoint tag: nothing to download offline. Seeded random weights only on
            # an explicit opt-in -- a filtered warning must never turn into silent
            # garbage accuracy (round-5 advice)
            if not allow_seeded:
                raise RuntimeError(
                    f"pretrained={pretrained!r} for {model_name}: no pretrained checkpoints are "
                    f"available offline. Pass a state-dict file path for real weights, or "
                    f"pretrained='seeded' / allow_seeded=True for SEEDED RANDOM weights.")
            warnings.warn(
                f"pretrained={pretrained!r} for {model_name}: no pretrained checkpoints are "
                f"available offline; loading SEEDED RANDOM weights (seed={seed}) of the "
                f"{model_name} shapes (allow_seeded=True).", SeededWeightsWarning, stacklevel=2)
        src, config = model_name, None
    with warnings.catch_warnings():
        # the tag warning above (or the explicit None / "seeded") already said it
        warnings.simplefilter("ignore", SeededWeightsWarning)
        _, model, _ = load(src, device=device, compute_dtype=compute_dtype, seed=seed,
                           surface="open_clip", config=config)
    return model


def create_model_and_transforms(model_name, pretrained=None, device="cuda", *,
                                compute_dtype="fp16", seed=0, **kwargs):
    from . import _transform
    model = create_model(model_name, pretrained, device, compute_dtype=compute_dtype, seed=seed,
                         **kwargs)
    pre = _transform(model.config.image_resolution)
    return model, pre, pre


def get_tokenizer(model_name=None):
    from . import tokenize

    def tok(texts, context_length: int = 77):
        # open_clip's tokenizer truncates over-long prompts (keeping the EOT token)
        return tokenize(texts, context_length=context_length, truncate=True)
    return tok


@torch.no_grad()
def encode_image_features(model, images, normalize=True):
    """What aihab_utils/feature_cache.py:124-128 stores per batch: post-projection
    (open_clip surface) embeddings, L2-normalised when asked, normalise fused."""
    return model.encode_image(images, normalize=normalize, apply_proj=True)
