"""The reference-side ctypes binding printed in INTEGRATION.md, executed as written.

INTEGRATION.md shows the stub a maintainer of the reference would add
(`clip/_miclip_ffi.py`: the miclip_config struct, miclip_model_create /
load_weights, and an `encode_image` patched onto the reference's CLIP object,
clip/model.py:238, 335-336). This test takes that code block verbatim (only the
library path is filled in), attaches it to an object with the reference CLIP's
attributes and state-dict names, and checks its features against the package's
own `encode_image` on the same seeded weights -- bit for bit, since both run the
same library with the default numerics. A stale struct layout or signature in
the document fails here.
"""
import os
import re
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    src = next(b for b in blocks if "_miclip_ffi.py" in b)
    lib = os.path.join(ROOT, "aihab-clip_amd", "miclip", "libmiclip.so")
    assert "/path/to/repo/aihab-clip_amd/miclip/libmiclip.so" in src
    return src.replace("/path/to/repo/aihab-clip_amd/miclip/libmiclip.so", lib)


def _reference_like(cfg, sd):
    """The attributes the stub reads from a reference CLIP (clip/model.py:238-290)."""
    tens = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}
    visual = SimpleNamespace(
        input_resolution=cfg.image_resolution,
        conv1=SimpleNamespace(weight=tens["visual.conv1.weight"]),
        transformer=SimpleNamespace(resblocks=[None] * cfg.vision_layers))
    return SimpleNamespace(visual=visual, context_length=cfg.context_length,
                           vocab_size=cfg.vocab_size,
                           transformer=SimpleNamespace(width=cfg.transformer_width,
                                                       layers=cfg.transformer_layers),
                           state_dict=lambda: tens)


@pytest.mark.parametrize("name", ["ViT-B/32", "ViT-B/16"])
def test_integration_stub_matches_package(name):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import miclip
    from miclip.configs import MODEL_CONFIGS
    from miclip.weights import generate_state_dict, synthetic_images
    cfg = MODEL_CONFIGS[name]
    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md:_miclip_ffi.py", "exec"), ns)
    ref_model = ns["attach"](_reference_like(cfg, generate_state_dict(cfg, seed=0)))
    imgs = torch.from_numpy(synthetic_images(5, cfg.image_resolution, seed=4)).cuda()
    got = ref_model.encode_image(imgs)
    got_h = ref_model.encode_image(imgs.half())
    _, m, _ = miclip.load(name, device="cuda")
    want = m.encode_image(imgs)
    torch.cuda.synchronize()
    assert got.shape == want.shape == (5, cfg.vision_width)
    assert torch.equal(got, want)
    assert torch.equal(got_h, m.encode_image(imgs.half()))
