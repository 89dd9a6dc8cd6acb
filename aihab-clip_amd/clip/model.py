"""`clip.model` drop-in names (clip/model.py:396 build_model, 238 CLIP)."""
from miclip.model import CLIP, build_model  # noqa: F401
