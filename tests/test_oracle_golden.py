"""CPU: the oracle (oracle/clip_oracle.py) against the reference goldens.

The goldens come from running the reference clip/model.py (build_model +
.float(), i.e. clip.load on CPU) in the build container; the oracle must
reproduce them on the same seeded inputs. This pins the oracle that the GPU
parity tests and smoke() check against.

Bit-exactness is a same-machine property: torch's fp32 CPU GEMM kernels pick
their blocking (and so their summation order) by CPU model and ISA, so the
fixtures (made on the round-1 Intel host) and an AMD EPYC host differ by
~2e-6 at |x| ~ 4. Against the committed fixtures the bound is therefore
CPU_TOL (fp32 reassociation, 5e-6 relative); when the reference is present
(the build container), test_oracle_bit_exact_vs_reference_here re-runs the
reference on THIS machine and requires the oracle to match it bit for bit.
"""
import os
import numpy as np
import pytest
import torch

from miclip.configs import MODEL_CONFIGS
from miclip.weights import generate_state_dict, synthetic_images, checksum
from oracle import clip_oracle

CPU_TOL = 2e-5     # max |d| vs fixtures made on another CPU (see module docstring)
REF = os.environ.get("MICLIP_REFERENCE", "/root/reference")

TAGS = {"vitb32": "ViT-B/32", "vitb16": "ViT-B/16", "vitl14": "ViT-L/14",
        "vitl14_336": "ViT-L/14@336px", "vith14": "ViT-H-14"}


@pytest.fixture(scope="module")
def states():
    cache = {}

    def get(name):
        if name not in cache:
            cache.clear()
            cache[name] = generate_state_dict(MODEL_CONFIGS[name], seed=0)
        return cache[name]
    return get


@pytest.mark.parametrize("tag", list(TAGS))
def test_generator_matches_fixture(golden, states, tag):
    g = golden(tag)
    sd = states(TAGS[tag])
    for name, crc in g["meta"]["weight_crc"].items():
        assert checksum(sd[name]) == crc, f"weight generator drifted for {name}"
    cfg = MODEL_CONFIGS[TAGS[tag]]
    imgs = synthetic_images(g["meta"]["n_images"], cfg.image_resolution, seed=0)
    assert checksum(imgs) == g["meta"]["image_crc"]


@pytest.mark.parametrize("tag", list(TAGS))
def test_goldens_are_discriminative(golden, tag):
    """The fixtures can tell one image from another: >= 16 structured images whose
    features differ by 1-cos >= 10x the 1e-3 parity tolerance between ANY two of
    them, an image-specific part of >= 30 % of the norm, and >= 3 distinct golden
    top-1 classes (the r01-r03 noise images shared ~95 % of their features and one
    top-1 class)."""
    g = golden(tag)
    f = torch.nn.functional.normalize(torch.from_numpy(g["image"]).double(), dim=-1)
    n = f.shape[0]
    inter = (1 - f @ f.T)[~torch.eye(n, dtype=torch.bool)]
    raw = torch.from_numpy(g["image"]).double()
    share = ((raw - raw.mean(0)).norm(dim=1) / raw.norm(dim=1)).mean().item()
    distinct = len(set(g["topk"][:, 0].tolist()))
    print(f"{tag}: {n} images, inter-image 1-cos min {inter.min():.3e}, specific share "
          f"{share:.2f}, {distinct} distinct top-1")
    assert g["meta"]["images"] == "structured" and n >= 16
    assert inter.min().item() >= 10 * 1e-3
    assert share >= 0.3 and distinct >= 3


@pytest.mark.parametrize("tag", ["vitb32", "vitb16", "vitl14", "vith14"])
def test_oracle_image_bit_exact(golden, states, tag):
    torch.set_num_threads(8)
    g = golden(tag)
    cfg = MODEL_CONFIGS[TAGS[tag]]
    sd = states(TAGS[tag])
    imgs = synthetic_images(g["meta"]["n_images"], cfg.image_resolution, seed=0)
    out = clip_oracle.encode_image(sd, cfg, imgs).numpy()
    assert np.abs(out - g["image"]).max() <= CPU_TOL


@pytest.mark.parametrize("tag", ["vitb32", "vitl14", "vith14"])
def test_oracle_text_and_head(golden, states, tag):
    g = golden(tag)
    cfg = MODEL_CONFIGS[TAGS[tag]]
    sd = states(TAGS[tag])
    xb, xp = clip_oracle.encode_text(sd, cfg, g["tokens"])
    assert np.abs(xb.numpy() - g["text_before"]).max() <= CPU_TOL
    assert np.abs(xp.numpy() - g["text_proj"]).max() <= CPU_TOL
    tw = clip_oracle.class_text_weights(sd, cfg, [t[None] for t in g["tokens"]])
    assert np.abs(tw.numpy() - g["text_weights"]).max() <= CPU_TOL
    logits = clip_oracle.zero_shot_logits(torch.from_numpy(g["image"]), sd["visual.proj"], tw)
    assert np.abs(logits.numpy() - g["logits"]).max() <= 1e-4
    assert np.array_equal(clip_oracle.topk(logits, g["topk"].shape[1]).numpy(), g["topk"])


def test_golden_tokens_well_formed(golden):
    for tag in ("vitb32", "vitl14"):
        tok = golden(tag)["tokens"]
        assert tok.shape[1] == 77 and (tok[:, 0] == 49406).all()
        eot = tok.argmax(axis=1)
        assert (tok[np.arange(len(tok)), eot] == 49407).all()
        assert all((row[e + 1:] == 0).all() for row, e in zip(tok, eot))


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "clip", "model.py")),
                    reason="reference checkout absent (only the build container has it)")
def test_oracle_bit_exact_vs_reference_here(golden):
    """Same machine, same torch: the oracle equals the reference clip/model.py
    (build_model + .float(), clip/clip.py:133-137) bit for bit -- image tower,
    text tuple and the clip_classifier / ProLIP head (oracle/make_golden.py)."""
    import sys
    sys.dont_write_bytecode = True
    from oracle import make_golden
    refmodel = make_golden._load("_ref_clip_model", os.path.join(REF, "clip", "model.py"))
    cfg = MODEL_CONFIGS["ViT-B/32"]
    sd = generate_state_dict(cfg, seed=0)
    model = make_golden.reference_model(refmodel, sd, cfg)
    imgs = synthetic_images(3, cfg.image_resolution, seed=0)
    tokens = golden("vitb32")["tokens"][:4]
    torch.set_num_threads(8)
    with torch.no_grad():
        ref_img = model.encode_image(torch.from_numpy(imgs))
        ref_b, ref_p = model.encode_text(torch.from_numpy(tokens).long())
    assert torch.equal(clip_oracle.encode_image(sd, cfg, imgs), ref_img)
    ob, op = clip_oracle.encode_text(sd, cfg, tokens)
    assert torch.equal(ob, ref_b) and torch.equal(op, ref_p)
