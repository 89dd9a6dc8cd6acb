"""`import open_clip` drop-in for the reference's open_clip path
(aihab_utils/model_init.py:42-112, methods/PEFT_openclip.py): with
`aihab-clip_amd/` first on sys.path, `open_clip.create_model_and_transforms`,
`open_clip.get_tokenizer` and `open_clip.create_model` resolve to miclip's
MI355X encode path (open_clip model surface).

Covered: the inference contract -- model_init, feature caching and eval. Not
covered: PEFT training (lock_image_tower / lock_text_tower and backward through
encode_image, methods/PEFT_openclip.py:197-273), which raises NotImplementedError.
`pretrained` must be a state-dict file or None / "seeded" (a checkpoint tag
raises: none are available offline)."""
from miclip.openclip import create_model, create_model_and_transforms, get_tokenizer, list_models  # noqa: F401

__all__ = ["create_model", "create_model_and_transforms", "get_tokenizer", "list_models"]
