"""`import clip` drop-in: the reference's call sites (aihab_utils/model_init.py:4,145;
utils.py:10,42) use `clip.load`, `clip.tokenize` and `clip.available_models`.
Putting `aihab-clip_amd/` first on sys.path makes those resolve to miclip's
MI355X encode path without editing the callers."""
from miclip import available_models, load, tokenize  # noqa: F401
from miclip import build_model  # noqa: F401

__all__ = ["available_models", "load", "tokenize"]
