"""On-device CLIP preprocessing against the reference transform.

The reference transform is torchvision over Pillow (clip/clip.py:74-81,
data/clip_transforms.py:50-55). torchvision is absent from this image; Pillow
(12.2.0) is present, so the checker is Pillow's own `Image.resize(BICUBIC)`
plus the torchvision size / crop-anchor / ToTensor / Normalize rules restated
in oracle/pil_resample.py. The numpy restatement of Resample.c in that file
is pinned against Pillow here (CPU). Bar: bit-exact, both for the uint8 crop
and for the float32 normalised tensor.
"""
import numpy as np
import pytest
import torch

from oracle import pil_resample as P

# (H, W, C): down/up-scaling, identity, portrait/landscape, odd sizes, 'L' images,
# a long side that truncates (int(n * long / short)), 1080p camera-trap frames.
SIZES = [(480, 640, 3), (300, 224, 3), (224, 224, 3), (100, 150, 3), (333, 517, 1),
         (224, 300, 3), (1200, 901, 3), (50, 60, 3), (225, 224, 3), (7, 9, 3), (1080, 1920, 3)]


def _image(rng, h, w, c, smooth=False):
    if smooth:      # natural-image-like gradients + texture (few clipped taps)
        y, x = np.mgrid[0:h, 0:w]
        base = 127 + 60 * np.sin(x / 17.0)[..., None] * np.cos(y / 23.0)[..., None]
        img = base + rng.normal(0, 20, (h, w, c))
        return np.clip(img, 0, 255).astype(np.uint8)
    return rng.integers(0, 256, (h, w, c), dtype=np.uint8)   # noise: worst case for clip8


# ---------------------------------------------------------------- CPU: the oracle
@pytest.mark.parametrize("n", [224, 336])
def test_restatement_matches_pillow(n):
    rng = np.random.default_rng(n)
    for h, w, c in SIZES[:-1]:
        img = _image(rng, h, w, c)
        a = P.crop_u8(img, n)
        b = P.crop_u8(img, n, resize=P.pil_resize)
        assert a.shape == (n, n, c) and np.array_equal(a, b), (h, w, c)


def test_torchvision_geometry_rules():
    assert P.output_size(480, 640, 224) == (224, 298)      # int(298.67): truncation
    assert P.output_size(640, 480, 224) == (298, 224)
    assert P.output_size(224, 224, 224) == (224, 224)
    assert P.output_size(1080, 1920, 336) == (336, 597)
    assert P.crop_anchor(224, 299, 224) == (0, 38)           # round(37.5) -> 38 (even)
    assert P.crop_anchor(224, 301, 224) == (0, 38)           # round(38.5) -> 38 (even)
    assert P.crop_anchor(224, 300, 224) == (0, 38)


def test_host_transform_matches_reference_rules():
    """miclip's host `preprocess` (returned by load) == Pillow + torchvision rules."""
    from PIL import Image
    from miclip.preprocess import Transform
    rng = np.random.default_rng(1)
    for h, w, c in [(480, 640, 3), (301, 224, 3), (333, 517, 1)]:
        img = _image(rng, h, w, c, smooth=True)
        pil = Image.fromarray(img if c == 3 else img[:, :, 0])
        got = Transform(224)(pil).numpy()
        ref = P.transform_reference(img, 224)
        assert np.array_equal(got, ref)


# ---------------------------------------------------------------- GPU: the kernel
def _tiny_model(n):
    import miclip
    from miclip.configs import CLIPConfig
    from miclip.weights import generate_state_dict
    cfg = CLIPConfig(embed_dim=64, image_resolution=n, vision_layers=1, vision_width=256,
                     vision_patch_size=n // 7, context_length=77, vocab_size=49408,
                     transformer_width=256, transformer_heads=4, transformer_layers=1)
    sd = {k: torch.from_numpy(v) for k, v in generate_state_dict(cfg, seed=0).items()}
    return miclip.CLIP(cfg, sd, device="cuda")


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [224, 336])
@pytest.mark.parametrize("smooth", [False, True])
def test_kernel_crop_bit_exact_ragged(gpu, n, smooth):
    rng = np.random.default_rng(7 + n)
    imgs = [_image(rng, h, w, c, smooth) for h, w, c in SIZES]
    m = _tiny_model(n)
    crops = m.preprocess_images(imgs, uint8=True).cpu().numpy()
    assert crops.shape == (len(imgs), n, n, 3)
    for i, img in enumerate(imgs):
        ref = P.to_rgb(P.crop_u8(img, n, resize=P.pil_resize))
        bad = np.argwhere(crops[i] != ref)
        assert bad.size == 0, (SIZES[i], bad[:5], crops[i][tuple(bad[0])], ref[tuple(bad[0])])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [224, 336])
def test_kernel_normalised_bit_exact(gpu, n):
    rng = np.random.default_rng(11)
    imgs = [_image(rng, h, w, c, smooth=True) for h, w, c in SIZES[:6]]
    m = _tiny_model(n)
    x = m.preprocess_images(imgs).cpu().numpy()
    assert x.dtype == np.float32 and x.shape == (len(imgs), 3, n, n)
    for i, img in enumerate(imgs):
        ref = P.transform_reference(img, n)
        assert np.array_equal(x[i], ref), (SIZES[i], np.abs(x[i] - ref).max())


@pytest.mark.gpu
def test_kernel_uniform_batch_device_tensor_and_stride(gpu):
    """[B,H,W,3] device tensor input == the same images as a list; large batch."""
    rng = np.random.default_rng(3)
    batch = np.stack([_image(rng, 375, 500, 3, smooth=True) for _ in range(40)])
    m = _tiny_model(224)
    a = m.preprocess_images(torch.from_numpy(batch).cuda())
    b = m.preprocess_images(list(batch))
    assert torch.equal(a, b)
    ref = P.transform_reference(batch[17], 224)
    assert np.array_equal(a[17].cpu().numpy(), ref)


@pytest.mark.gpu
def test_kernel_rejects_bad_input(gpu):
    m = _tiny_model(224)
    with pytest.raises(ValueError):
        m.preprocess_images([np.zeros((32, 32, 4), np.uint8)])       # RGBA not supported
    with pytest.raises(ValueError):
        m.preprocess_images([np.zeros((32, 32, 3), np.float32)])
    with pytest.raises(ValueError):
        m.preprocess_images([np.zeros((4000, 4000, 1), np.uint8)])   # > 64 taps per pass
    assert m.preprocess_images([]).shape == (0, 3, 224, 224)


@pytest.mark.gpu
def test_device_preprocess_feeds_encode_image_identically(gpu):
    """encode_image(device preprocess) == encode_image(reference host transform), bitwise."""
    import miclip
    from PIL import Image
    rng = np.random.default_rng(5)
    imgs = [_image(rng, h, w, 3, smooth=True) for h, w in [(480, 640), (300, 400), (256, 256)]]
    _, model, preprocess = miclip.load("ViT-B/32", device="cuda")
    host = torch.stack([preprocess(Image.fromarray(a)) for a in imgs]).cuda()
    dev = model.preprocess_images(imgs)
    assert torch.equal(host, dev)
    assert torch.equal(model.encode_image(host), model.encode_image(dev))
