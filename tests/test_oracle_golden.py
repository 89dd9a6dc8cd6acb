"""CPU: the oracle (oracle/clip_oracle.py) against the reference goldens.

The goldens come from running the reference clip/model.py (build_model +
.float(), i.e. clip.load on CPU) in the build container; the oracle must
reproduce them bit-exactly on the same seeded inputs. This pins the oracle
that the GPU parity tests and smoke() check against.
"""
import numpy as np
import pytest
import torch

from miclip.configs import MODEL_CONFIGS
from miclip.weights import generate_state_dict, synthetic_images, checksum
from oracle import clip_oracle

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


@pytest.mark.parametrize("tag", ["vitb32", "vitb16", "vitl14", "vith14"])
def test_oracle_image_bit_exact(golden, states, tag):
    torch.set_num_threads(8)
    g = golden(tag)
    cfg = MODEL_CONFIGS[TAGS[tag]]
    sd = states(TAGS[tag])
    imgs = synthetic_images(g["meta"]["n_images"], cfg.image_resolution, seed=0)
    out = clip_oracle.encode_image(sd, cfg, imgs).numpy()
    assert np.abs(out - g["image"]).max() <= 1e-6


@pytest.mark.parametrize("tag", ["vitb32", "vitl14", "vith14"])
def test_oracle_text_and_head(golden, states, tag):
    g = golden(tag)
    cfg = MODEL_CONFIGS[TAGS[tag]]
    sd = states(TAGS[tag])
    xb, xp = clip_oracle.encode_text(sd, cfg, g["tokens"])
    assert np.abs(xb.numpy() - g["text_before"]).max() <= 1e-6
    assert np.abs(xp.numpy() - g["text_proj"]).max() <= 1e-6
    tw = clip_oracle.class_text_weights(sd, cfg, [t[None] for t in g["tokens"]])
    assert np.abs(tw.numpy() - g["text_weights"]).max() <= 1e-6
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
