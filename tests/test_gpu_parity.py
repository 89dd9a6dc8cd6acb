"""End-to-end parity of the HIP encode path against the reference goldens.

Goldens (tests/golden/*.npz) were produced by running the reference
clip/model.py on CPU in fp32 (oracle/make_golden.py). Here the same seeded
weights and inputs go through `miclip.load(...)` -> C ABI -> HIP kernels.

Tolerances (north_star / SURVEY §8c):
  * embeddings: 1 - cos <= 1e-3 per row (image pre-projection features,
    text x_before and x), and the same bound on the CENTRED image features
    (each set minus its mean: only the image-specific part; tests/_parity.py).
    The goldens hold 16 structured images per config whose features differ by
    1-cos >= 1.1e-2 between any two images (>= 10x the tolerance, printed);
  * zero-shot top-1: bit-exact on every row whose golden top1-top2 margin
    exceeds the logit error bound measured on that same run (2 x max |dlogit|);
    rows inside the bound are reported, not asserted (random-init CLIP has
    near-tied logits; SURVEY §7 "Hard parts"). The golden top-1 column holds
    >= 3 distinct classes per config, and the number of asserted rows is printed.
"""
import numpy as np
import pytest
import torch

from _parity import one_minus_cos, report, top1_report

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3
CONFIGS = [("vitb32", "ViT-B/32"), ("vitb16", "ViT-B/16"), ("vitl14", "ViT-L/14"),
           ("vitl14_336", "ViT-L/14@336px"), ("vith14", "ViT-H-14")]


_one_minus_cos = one_minus_cos


_models = {}


def _model(name, dtype):
    import miclip
    key = (name, dtype)
    if key not in _models:
        _models.clear()
        torch.cuda.empty_cache()
        # the vendored OpenAI surface (pre-projection image features, tuple
        # encode_text) for every name, ViT-H-14 included: the goldens hold the
        # pre-projection features (open_clip surface: test_gpu_openclip.py)
        _, m, _ = miclip.load(name, device="cuda", compute_dtype=dtype, surface="openai")
        _models[key] = m
    return _models[key]


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    yield
    _models.clear()


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
@pytest.mark.parametrize("tag,name", CONFIGS)
def test_encode_image_matches_reference(golden, tag, name, dtype):
    from miclip.configs import MODEL_CONFIGS
    from miclip.weights import synthetic_images, checksum
    g = golden(tag)
    cfg = MODEL_CONFIGS[name]
    imgs = synthetic_images(g["meta"]["n_images"], cfg.image_resolution, seed=g["meta"]["seed"])
    assert checksum(imgs) == g["meta"]["image_crc"], "synthetic image generator drifted"
    m = _model(name, dtype)
    feats = m.encode_image(torch.from_numpy(imgs).cuda()).cpu()
    assert feats.shape == g["image"].shape and feats.dtype == torch.float32
    report(f"{tag}/{dtype}", feats, g["image"], COS_TOL, COS_TOL)


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
def test_fp32_residual_stream_option(golden, dtype):
    """options={"resid_f32": True} keeps an fp32 residual stream (the default streams
    fp16 under fp16 and bf16 compute, like the reference's GPU model); both meet the
    tolerance, raw and centred, and the text tower follows the same option."""
    import miclip
    from miclip.weights import synthetic_images
    g = golden("vitb16")
    imgs = torch.from_numpy(synthetic_images(g["meta"]["n_images"], 224, seed=0)).cuda()
    _models.clear()
    _, m32, _ = miclip.load("ViT-B/16", device="cuda", compute_dtype=dtype,
                            options={"resid_f32": True})
    assert not m32.numerics()["resid16"]
    f32 = m32.encode_image(imgs).cpu()
    t32 = m32.encode_text(torch.from_numpy(g["tokens"]).long().cuda())[1].cpu()
    del m32
    m16 = _model("ViT-B/16", dtype)
    assert m16.numerics()["resid16"]
    assert m16.numerics()["lnfold"] == (dtype == "fp16")
    f16 = m16.encode_image(imgs).cpu()
    t16 = m16.encode_text(torch.from_numpy(g["tokens"]).long().cuda())[1].cpu()
    report(f"vitb16/{dtype} fp32 stream", f32, g["image"], COS_TOL, COS_TOL)
    report(f"vitb16/{dtype} fp16 stream", f16, g["image"], COS_TOL, COS_TOL)
    dt32, dt16 = _one_minus_cos(t32, g["text_proj"]), _one_minus_cos(t16, g["text_proj"])
    print(f"vitb16/{dtype}: text 1-cos fp32 stream {dt32.max():.2e}, fp16 stream {dt16.max():.2e}")
    assert dt32.max() <= COS_TOL and dt16.max() <= COS_TOL
    assert not torch.equal(f32, f16), "the option did not change the stream"


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
@pytest.mark.parametrize("tag,name", CONFIGS[:3] + CONFIGS[4:])
def test_encode_text_matches_reference(golden, tag, name, dtype):
    g = golden(tag)
    m = _model(name, dtype)
    xb, xp = m.encode_text(torch.from_numpy(g["tokens"]).long().cuda())
    d1 = _one_minus_cos(xb.cpu(), g["text_before"])
    d2 = _one_minus_cos(xp.cpu(), g["text_proj"])
    print(f"{tag}/{dtype}: text 1-cos max before {d1.max():.2e} proj {d2.max():.2e}")
    assert d1.max() <= COS_TOL and d2.max() <= COS_TOL


def test_vitl14_336_text_golden_is_vitl14s(golden):
    """test_encode_text_matches_reference skips vitl14_336 because its text tower is
    ViT-L/14's (same text config and seeded weights): the two goldens must stay
    byte-identical, or a regeneration could silently drop C4's text check."""
    a, b = golden("vitl14"), golden("vitl14_336")
    for key in ("tokens", "text_before", "text_proj", "text_weights"):
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.parametrize("tag,name", CONFIGS)
def test_zero_shot_top1(golden, tag, name):
    """Full chain on the GPU: encode_image -> proj -> normalize -> 100*f@W -> topk."""
    from miclip.configs import MODEL_CONFIGS
    from miclip.weights import synthetic_images
    g = golden(tag)
    m = _model(name, "fp16")
    imgs = synthetic_images(g["meta"]["n_images"], MODEL_CONFIGS[name].image_resolution, seed=0)
    feats = m.encode_image(torch.from_numpy(imgs).cuda())
    tw = torch.from_numpy(g["text_weights"]).cuda()
    logits, top = m.zero_shot(feats, tw, scale=100.0, k=g["topk"].shape[1])
    logits, top = logits.cpu().numpy(), top.cpu().numpy()
    err = np.abs(logits - g["logits"]).max()
    bound = 2 * err
    sure = g["margins"] > bound
    print(f"{tag}: max|dlogit| {err:.4f}, golden margins {np.round(np.sort(g['margins'])[:4], 3)}..")
    assert err < 1.0
    top1_report(tag, top[:, 0], g["topk"][:, 0], sure)


def test_zero_shot_head_exact_on_reference_features(golden):
    """The head alone, fed the golden fp32 features: logits within fp32 rounding,
    top-k indices bit-exact (no near ties at that precision)."""
    g = golden("vitl14")
    m = _model("ViT-L/14", "fp16")
    logits, top = m.zero_shot(torch.from_numpy(g["image"]).cuda(),
                              torch.from_numpy(g["text_weights"]).cuda(), 100.0, k=5)
    assert np.abs(logits.cpu().numpy() - g["logits"]).max() < 1e-3
    assert np.array_equal(top.cpu().numpy(), g["topk"])


def test_batch_invariance_and_shards():
    """Size-independent property at a bench-like batch: encoding a batch equals
    encoding its shards (row order preserved), so the sharded feature cache is
    exactly the single-GPU cache."""
    from miclip.weights import synthetic_images
    m = _model("ViT-B/32", "fp16")
    # two streams from 2 x 4096 token rows and 2 x 16 images (capi.hip image_splits):
    # the 192-image batch runs split, its 32-image shards on one stream
    m.set_splits(2)
    assert m.image_splits(96) == 1 and m.image_splits(192) == 2 and m.image_splits(32) == 1
    imgs = torch.from_numpy(synthetic_images(192, 224, seed=3)).cuda()
    full = m.encode_image(imgs)
    parts = torch.cat([m.encode_image(imgs[i:i + 32]) for i in range(0, 192, 32)])
    assert torch.equal(full, parts)
    again = m.encode_image(imgs)
    assert torch.equal(full, again), "encode is not deterministic"


@pytest.mark.parametrize("name,dtype,tol", [("ViT-B/16", "fp16", 2e-5), ("ViT-B/32", "bf16", 2e-4),
                                            ("ViT-L/14", "fp16", 2e-5), ("ViT-H-14", "mxfp8", 1e-3)])
def test_cls_last_block_matches_full(name, dtype, tol):
    """The last vision block on the CLS rows only (default) against the whole
    block (set_cls_last(False), MICLIP_OPT_FULL_LAST_BLOCK): the same features up
    to the CLS attention's summation order (VALU dot products vs MFMA tiles)."""
    from miclip.weights import synthetic_images
    m = _model(name, dtype)
    imgs = torch.from_numpy(synthetic_images(6, 224, seed=5)).cuda()
    fast = m.encode_image(imgs).float().cpu()
    assert m.numerics()["cls_last"]
    m.set_cls_last(False)
    try:
        assert not m.numerics()["cls_last"]
        full = m.encode_image(imgs).float().cpu()
    finally:
        m.set_cls_last(True)
    d = 1 - torch.nn.functional.cosine_similarity(fast, full, dim=1)
    print(f"{name} {dtype}: 1-cos max {d.max().item():.2e}")
    assert d.max().item() <= tol


def test_normalize_and_proj_flags(golden):
    g = golden("vitb32")
    from miclip.weights import synthetic_images
    m = _model("ViT-B/32", "fp16")
    imgs = torch.from_numpy(synthetic_images(8, 224, seed=0)).cuda()
    raw = m.encode_image(imgs)
    nrm = m.encode_image(imgs, normalize=True)
    assert torch.allclose(nrm, torch.nn.functional.normalize(raw, dim=-1), atol=1e-6)
    prj = m.encode_image(imgs, apply_proj=True)
    ref = raw @ m.visual.proj
    assert torch.allclose(prj, ref, rtol=1e-4, atol=1e-4)
    both = m.encode_image(imgs, normalize=True, apply_proj=True)
    assert torch.allclose(both, torch.nn.functional.normalize(ref, dim=-1), atol=1e-5)


def test_edge_batches():
    m = _model("ViT-B/32", "fp16")
    from miclip.weights import synthetic_images
    one = torch.from_numpy(synthetic_images(1, 224, seed=5)).cuda()
    assert m.encode_image(one).shape == (1, 768)
    empty = torch.empty(0, 3, 224, 224, device="cuda")
    assert m.encode_image(empty).shape == (0, 768)
    with pytest.raises(ValueError):
        m.encode_image(torch.zeros(2, 3, 225, 225, device="cuda"))
    with pytest.raises(ValueError):
        m.encode_text(torch.zeros(2, 76, dtype=torch.long, device="cuda"))
    with pytest.raises(IndexError):
        m.encode_text(torch.full((1, 77), 49408, dtype=torch.long))


def test_runtime_toggles_survive_device_moves():
    """set_cls_last / set_splits are runtime settings of the C handle; a device move
    rebuilds the handle from the module, which must re-apply them (round-4 advice)."""
    from miclip.weights import synthetic_images
    m = _model("ViT-B/32", "fp16")
    imgs = torch.from_numpy(synthetic_images(3, 224, seed=9)).cuda()
    m.set_cls_last(False)
    m.set_splits(1)
    try:
        full = m.encode_image(imgs)
        m.cpu()
        m.cuda()
        assert not m.numerics()["cls_last"]
        assert torch.equal(m.encode_image(imgs), full)
    finally:
        m.set_cls_last(True)
        m.set_splits(2)
    assert m.numerics()["cls_last"]


def test_module_surface():
    m = _model("ViT-B/32", "fp16")
    sd = m.state_dict()
    assert sd["visual.proj"].shape == (768, 512)
    assert next(m.parameters()).device.type == "cuda"
    assert m.visual.input_resolution == 224 and m.dtype == torch.float16
    assert "visual.transformer.resblocks.11.mlp.c_proj.weight" in sd


@pytest.mark.parametrize("B,C,k", [(13, 20, 5), (1, 7, 1), (64, 1000, 5), (256, 1000, 10),
                                   (17, 16, 16), (40, 33, 3)])
def test_zero_shot_head_vs_torch(B, C, k):
    """The head on the f32 MFMA (16 x 16 logits tiles, normalise fused; ragged rows and
    classes) and the top-k kernel against torch fp32."""
    m = _model("ViT-B/32", "fp16")
    g = torch.Generator(device="cuda").manual_seed(B + C)
    feats = torch.randn(B, 768, device="cuda", generator=g)
    tw = torch.nn.functional.normalize(torch.randn(512, C, device="cuda", generator=g), dim=0)
    logits, top = m.zero_shot(feats, tw, 100.0, k=k, apply_proj=True)
    ref = 100.0 * torch.nn.functional.normalize(feats @ m.visual.proj, dim=-1) @ tw
    assert (logits - ref).abs().max().item() < 2e-3
    rv, ri = ref.topk(k, 1, True, True)
    gap = (rv[:, :-1] - rv[:, 1:]).min().item() if k > 1 else 1.0
    if gap > 1e-3:
        assert torch.equal(top.cpu(), ri.cpu())
    nf = torch.nn.functional.normalize(feats @ m.visual.proj, dim=-1)
    l2, _ = m.zero_shot(nf, tw, 100.0, k=0, apply_proj=False)
    assert (l2 - ref).abs().max().item() < 2e-3


# MICLIP_MXFP8: parity unpinned with respect to the
# reference (no fp8 path there). The vision tower runs MX-fp8 GEMMs and is held
# to the north star's 1e-3 like every other path (measured 7.3e-4 ViT-H-14, 8.2e-4
# ViT-B/32, profiles/r05/configs/parity.log); the centred figure -- the image-
# specific part of the feature, which fp8 perturbs ~10x more than fp16 -- stays
# bounded at 1e-2 and printed. The text tower runs fp16 under mxfp8.
MX_COS_TOL_IMAGE = 1e-3
MX_CENTRED_TOL_IMAGE = 1e-2
MX_COS_TOL_TEXT = COS_TOL


@pytest.mark.parametrize("tag,name", [("vitb32", "ViT-B/32"), ("vith14", "ViT-H-14")])
def test_mxfp8_encode_within_fp8_tolerance(golden, tag, name):
    from miclip.configs import MODEL_CONFIGS
    from miclip.weights import synthetic_images
    g = golden(tag)
    imgs = synthetic_images(g["meta"]["n_images"], MODEL_CONFIGS[name].image_resolution, seed=0)
    m = _model(name, "mxfp8")
    feats = m.encode_image(torch.from_numpy(imgs).cuda()).cpu()
    report(f"{tag}/mxfp8", feats, g["image"], MX_COS_TOL_IMAGE, MX_CENTRED_TOL_IMAGE)
    nm = m.numerics()
    # the MX vision tower is not LN-folded; the fp16 text tower is (round-4 advice)
    assert nm["mxfp8"] and not nm["lnfold"] and nm["lnfold_text"]
    xb, xp = m.encode_text(torch.from_numpy(g["tokens"]).long().cuda())
    db = _one_minus_cos(xb.cpu(), g["text_before"])
    dt = _one_minus_cos(xp.cpu(), g["text_proj"])
    print(f"{tag}/mxfp8: text (fp16 tower) 1-cos max before {db.max():.2e} proj {dt.max():.2e}")
    assert db.max() <= MX_COS_TOL_TEXT and dt.max() <= MX_COS_TOL_TEXT
