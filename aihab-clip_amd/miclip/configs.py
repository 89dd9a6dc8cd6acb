"""Model shape table for the CLIP ViT dual encoder.

Shapes follow the hyper-parameter inference rules of the reference
`build_model` (clip/model.py:396-419) and the `CLIP` constructor
(clip/model.py:257-290): heads = width // 64, MLP = 4 * width,
tokens N = (R // P)**2 + 1, text context 77, vocab 49408.

No checkpoints exist offline, so model *names* resolve to these shapes with
seeded random weights (see `weights.py`); file paths go through
`config_from_state_dict`, the restatement of build_model's shape inference.
"""
from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class CLIPConfig:
    embed_dim: int
    image_resolution: int
    vision_layers: int
    vision_width: int
    vision_patch_size: int
    context_length: int
    vocab_size: int
    transformer_width: int
    transformer_heads: int
    transformer_layers: int
    # "quick" = x*sigmoid(1.702x) (OpenAI CLIP, clip/model.py:160-162);
    # "erf" = exact GELU (open_clip ViT-H/14 shapes, stretch config C5).
    act: str = "quick"
    # Vision head width: 64 in every OpenAI CLIP (clip/model.py:268 heads = width // 64);
    # open_clip's ViT-H/14 runs 16 heads of 80 on width 1280.
    vision_head_width: int = 64

    @property
    def vision_heads(self) -> int:
        # clip/model.py:268 (head_width 64); open_clip model configs name it directly
        return self.vision_width // self.vision_head_width

    @property
    def grid(self) -> int:
        return self.image_resolution // self.vision_patch_size

    @property
    def n_tokens(self) -> int:
        return self.grid * self.grid + 1

    @property
    def patch_dim(self) -> int:
        return 3 * self.vision_patch_size * self.vision_patch_size

    def to_dict(self):
        return asdict(self)


_TEXT_512 = dict(context_length=77, vocab_size=49408, transformer_width=512,
                 transformer_heads=8, transformer_layers=12)
_TEXT_768 = dict(context_length=77, vocab_size=49408, transformer_width=768,
                 transformer_heads=12, transformer_layers=12)

MODEL_CONFIGS = {
    "ViT-B/32": CLIPConfig(embed_dim=512, image_resolution=224, vision_layers=12,
                           vision_width=768, vision_patch_size=32, **_TEXT_512),
    "ViT-B/16": CLIPConfig(embed_dim=512, image_resolution=224, vision_layers=12,
                           vision_width=768, vision_patch_size=16, **_TEXT_512),
    "ViT-L/14": CLIPConfig(embed_dim=768, image_resolution=224, vision_layers=24,
                           vision_width=1024, vision_patch_size=14, **_TEXT_768),
    "ViT-L/14@336px": CLIPConfig(embed_dim=768, image_resolution=336, vision_layers=24,
                                 vision_width=1024, vision_patch_size=14, **_TEXT_768),
    # open_clip "ViT-H-14" shapes (stretch config C5; the reference
    # loads it through aihab_utils/model_init.py:42-112): same dual-encoder graph as
    # OpenAI CLIP with exact-erf GELU in the MLPs and 80-wide vision heads.
    "ViT-H-14": CLIPConfig(embed_dim=1024, image_resolution=224, vision_layers=32,
                           vision_width=1280, vision_patch_size=14, context_length=77,
                           vocab_size=49408, transformer_width=1024, transformer_heads=16,
                           transformer_layers=24, act="erf", vision_head_width=80),
}


# Names whose reference loader is open_clip (aihab_utils/model_init.py:42-112), so
# miclip.load gives them open_clip's model surface by default (model.py).
OPEN_CLIP_MODELS = frozenset({"ViT-H-14"})


def available_models():
    """Counterpart of clip.available_models (clip/clip.py:84-86), ViT names only."""
    return list(MODEL_CONFIGS.keys())


def config_from_state_dict(state_dict) -> CLIPConfig:
    """Shape inference of reference build_model (clip/model.py:396-419), ViT branch.

    ResNet checkpoints (no "visual.proj") are out of scope
    and raise ValueError.
    """
    if "visual.proj" not in state_dict:
        raise ValueError("only ViT CLIP checkpoints are supported (no 'visual.proj' key)")
    shape = lambda k: tuple(state_dict[k].shape)
    vision_width = shape("visual.conv1.weight")[0]
    vision_layers = len([k for k in state_dict
                         if k.startswith("visual.") and k.endswith(".attn.in_proj_weight")])
    vision_patch_size = shape("visual.conv1.weight")[-1]
    grid_size = round((shape("visual.positional_embedding")[0] - 1) ** 0.5)
    image_resolution = vision_patch_size * grid_size
    embed_dim = shape("text_projection")[1]
    context_length = shape("positional_embedding")[0]
    vocab_size = shape("token_embedding.weight")[0]
    transformer_width = shape("ln_final.weight")[0]
    transformer_heads = transformer_width // 64
    transformer_layers = len(set(k.split(".")[2] for k in state_dict
                                 if k.startswith("transformer.resblocks")))
    return CLIPConfig(embed_dim=embed_dim, image_resolution=image_resolution,
                      vision_layers=vision_layers, vision_width=vision_width,
                      vision_patch_size=vision_patch_size, context_length=context_length,
                      vocab_size=vocab_size, transformer_width=transformer_width,
                      transformer_heads=transformer_heads,
                      transformer_layers=transformer_layers)


def algorithmic_gflop_per_image(cfg: CLIPConfig) -> float:
    """F = 2*n*3P^2*W + L*(24*N*W^2 + 4*N^2*W), n = N-1 patches.

    Counts every GEMM and both attention matmuls of encode_image, no final proj.
    """
    W, L, N, P = cfg.vision_width, cfg.vision_layers, cfg.n_tokens, cfg.vision_patch_size
    n = N - 1
    return (2 * n * 3 * P * P * W + L * (24 * N * W * W + 4 * N * N * W)) / 1e9


def executed_gflop_per_image(cfg: CLIPConfig, cls_last: bool = True) -> float:
    """FLOPs encode_image's kernels execute per image. With the last vision block
    on the CLS rows only (capi.hip run_block(cls_only), default; its other rows
    never reach ln_post(x[:, 0, :]), clip/model.py:226-229) that block runs its QKV
    GEMM over all N rows (keys / values) but attention for one query and
    out-proj + MLP on one row: 6NW^2 + 4NW + 18W^2 instead of 24NW^2 + 4N^2W."""
    full = algorithmic_gflop_per_image(cfg)
    if not cls_last:
        return full
    W, N = cfg.vision_width, cfg.n_tokens
    layer = 24 * N * W * W + 4 * N * N * W
    last = 6 * N * W * W + 4 * N * W + 18 * W * W
    return full - (layer - last) / 1e9
