"""CPU: host-side logic of the drop-in surface (no kernels run here)."""
import os

import numpy as np
import pytest
import torch

import miclip
from miclip.configs import MODEL_CONFIGS, config_from_state_dict, algorithmic_gflop_per_image
from miclip.feature_cache import (_canonical_backbone_name, _embedding_cache_dir,
                                  _feature_cache_dir, _feature_cache_exists, shard_range)
from miclip.weights import param_specs

REF_BPE = "/root/reference/clip/bpe_simple_vocab_16e6.txt.gz"


# build_model's shape inference (clip/model.py:396-419) only covers OpenAI CLIP
# checkpoints; the open_clip ViT-H-14 entry (GELU, 80-wide heads) is name-only.
@pytest.mark.parametrize("name", [n for n, c in MODEL_CONFIGS.items() if c.act == "quick"])
def test_config_inference_roundtrip(name):
    cfg = MODEL_CONFIGS[name]
    fake = {n: np.empty(shape, dtype=np.float32) for n, shape, _, _ in param_specs(cfg)}
    assert config_from_state_dict(fake) == cfg


def test_resnet_checkpoints_rejected():
    with pytest.raises(ValueError):
        config_from_state_dict({"visual.layer1.0.conv1.weight": np.empty((64, 64, 1, 1))})


def test_load_errors_like_reference():
    with pytest.raises(RuntimeError, match="not found; available models"):
        miclip.load("RN50x64-not-a-model", device="cuda")


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_product_path_has_no_cpu_fallback():
    with pytest.raises(RuntimeError, match="HIP"):
        miclip.load("ViT-B/32", device="cpu")


def test_flop_model_matches_survey():
    # 8.82 / 162.02 / 381.92 GFLOP per image
    assert abs(algorithmic_gflop_per_image(MODEL_CONFIGS["ViT-B/32"]) - 8.82) < 0.01
    assert abs(algorithmic_gflop_per_image(MODEL_CONFIGS["ViT-L/14"]) - 162.02) < 0.01
    assert abs(algorithmic_gflop_per_image(MODEL_CONFIGS["ViT-L/14@336px"]) - 381.92) < 0.01


def test_cache_paths_match_reference_layout(tmp_path):
    cfg = {"root_path": str(tmp_path), "clip_backend": "openai", "backbone": "ViT-B/32",
           "dataset": "cs", "shots": 0, "seed": 1, "finetune": {}}
    assert _feature_cache_dir(cfg) == tmp_path / "features_ViTB32_cs" / "0_shot" / "seed1"
    assert _embedding_cache_dir(cfg, "Test") == tmp_path / "feat_cache_vis" / "ViTB32_cs" / "test" / "seed1"
    assert _canonical_backbone_name("hf-hub:timm/ViT-SO400M-14-SigLIP") == "hf-hub_timm_ViT-SO400M-14-SigLIP"
    d = _feature_cache_dir(cfg)
    assert not _feature_cache_exists(d, 2)
    d.mkdir(parents=True)
    for f in ("label.pth", "f0.pth", "f1.pth"):
        (d / f).write_bytes(b"x")
    assert _feature_cache_exists(d, 2) and not _feature_cache_exists(d, 3)


@pytest.mark.parametrize("n,world", [(256, 8), (7, 2), (1, 2), (0, 4), (255, 8)])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    sizes = [hi - lo for lo, hi in spans]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.skipif(not os.path.isfile(REF_BPE), reason="BPE vocabulary not available")
def test_tokenizer_matches_reference_tokens(golden, monkeypatch):
    monkeypatch.setenv("MICLIP_BPE_PATH", REF_BPE)
    import miclip.tokenizer as tk
    tk._tok = None
    for tag in ("vitb32", "vitl14"):
        g = golden(tag)
        got = miclip.tokenize(g["meta"]["prompts"])
        assert np.array_equal(got.numpy(), g["tokens"].astype(np.int64))
    with pytest.raises(RuntimeError, match="too long"):
        miclip.tokenize("word " * 100)
    t = miclip.tokenize("word " * 100, truncate=True)
    assert t.shape == (1, 77) and t[0, -1] == 49407


def test_preprocess_shapes():
    from PIL import Image
    _, _, pre = None, None, miclip._transform(224)
    img = Image.fromarray((np.random.default_rng(0).random((300, 400, 3)) * 255).astype(np.uint8))
    x = pre(img)
    assert x.shape == (3, 224, 224) and x.dtype == torch.float32
    assert -2.5 < float(x.min()) and float(x.max()) < 2.7


def test_openclip_pretrained_rules():
    """open_clip.create_model: a checkpoint tag (no checkpoints offline) raises unless
    the caller opts in (allow_seeded=True), and then loads the seeded weights with a
    SeededWeightsWarning -- never silently (round-5 advice); an unknown model
    raises like open_clip; a state-dict file is checked against the NAMED config
    (ViT-H-14: GELU, 80-wide heads), which build_model's inference cannot see."""
    from types import SimpleNamespace
    from miclip import _checked_config
    import miclip
    from miclip.openclip import create_model
    captured = {}

    def fake_load(src, **kw):
        captured.update(src=src, **kw)
        raise RuntimeError("stop before the GPU")
    real = miclip.load
    miclip.load = fake_load
    try:
        for tag in ("openai", "laion2b_s32b_b79k"):
            with pytest.raises(RuntimeError, match="no pretrained checkpoints"):
                create_model("ViT-H-14", pretrained=tag, device="cpu")
            assert not captured
            with pytest.warns(miclip.SeededWeightsWarning, match="SEEDED RANDOM"):
                with pytest.raises(RuntimeError, match="stop before the GPU"):
                    create_model("ViT-H-14", pretrained=tag, device="cpu", allow_seeded=True)
            assert captured["src"] == "ViT-H-14" and captured["config"] is None
            captured.clear()
        with pytest.raises(RuntimeError, match="stop before the GPU"):
            create_model("ViT-H-14", pretrained="seeded", device="cpu")
    finally:
        miclip.load = real
    with pytest.raises(RuntimeError, match="not found"):
        create_model("ViT-Q-99")
    cfg = MODEL_CONFIGS["ViT-H-14"]
    sd = {k: SimpleNamespace(shape=s) for k, s, _, _ in param_specs(cfg)}
    assert _checked_config("ViT-H-14", sd, "f.pt") is cfg
    inferred = config_from_state_dict(sd)
    assert inferred.act == "quick" and cfg.act == "erf"      # why the named config is needed
    sd["visual.proj"] = SimpleNamespace(shape=(1280, 768))
    with pytest.raises(RuntimeError, match="visual.proj has shape"):
        _checked_config("ViT-H-14", sd, "f.pt")


def test_numerics_options_are_explicit():
    """Every results-changing path is a named load() option (MICLIP_OPT_* bits);
    the HIP library reads no environment variables."""
    import re
    from miclip.model import OPTIONS, option_bits
    from miclip import _lib
    assert option_bits(None) == 0 and option_bits({"ln_fold": True, "cls_last": True}) == 0
    assert option_bits({"resid_f32": True}) == _lib.MICLIP_OPT_RESID_F32
    assert option_bits({"ln_fold": False, "cls_last": False}) == (
        _lib.MICLIP_OPT_NO_LN_FOLD | _lib.MICLIP_OPT_FULL_LAST_BLOCK)
    with pytest.raises(ValueError, match="unknown miclip option"):
        option_bits({"fast": True})
    csrc = os.path.join(os.path.dirname(miclip.__file__), "..", "csrc")
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        assert not re.search(r"\bgetenv\s*\(", text), f"{f} reads the environment"
