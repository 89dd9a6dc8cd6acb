"""The other BASELINE configs at their benched batch sizes, pinned to the goldens.

The goldens hold 2-8 images, which alone run tiny GEMMs (M = a few hundred rows,
no stream split, no row tails). Here each config runs at the batch its bench
line uses, with the golden images placed at the first row, either side of the
stream split and the last row, so the production launch shapes meet the
reference (as tests/test_gpu_lnfold.py:test_benched_config_vitl14_bs256 does
for C3):

  C2  ViT-B/32 bf16, bs=256: 2 streams of M = 6 400 (N = 768 tile columns)
  C4  ViT-L/14@336px fp16, bs=256: 2 streams of M = 73 856, attention at
      N = 577 (one head per workgroup), row tails
  C5  ViT-H-14 mxfp8, bs=512: MX-fp8 GEMMs over 2 streams of M = 65 792,
      head dim 80 (open_clip shapes; OpenAI surface: pre-projection goldens)

Each golden row must be within the config's tolerance of the reference
(1-cos <= 1e-3, MX-fp8 included; its centred bound 1e-2, tests/test_gpu_parity.py)
and bitwise equal to the small-batch encode of the same images (batch
invariance: the GEMM tiles, tails and splits keep one k order). A half-precision
input batch in the compute dtype (miclip_encode_image_ex) gives the same
features bit for bit (the patchify rounds pixels to the compute dtype anyway).
Reference: clip/model.py:216-235.
"""
import numpy as np
import pytest
import torch

from _parity import centred_one_minus_cos

pytestmark = pytest.mark.gpu


def _one_minus_cos(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return (1 - torch.nn.functional.cosine_similarity(a, b, dim=-1)).numpy()


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    yield
    torch.cuda.empty_cache()


@pytest.mark.parametrize("tag,name,dtype,bs,splits,tol,ctol", [
    ("vitb32", "ViT-B/32", "bf16", 256, 2, 1e-3, 1e-3),
    ("vitl14_336", "ViT-L/14@336px", "fp16", 256, 2, 1e-3, 1e-3),
    ("vith14", "ViT-H-14", "mxfp8", 512, 2, 1e-3, 1e-2),
])
def test_large_batch_config(golden, tag, name, dtype, bs, splits, tol, ctol):
    import miclip
    from miclip.configs import MODEL_CONFIGS
    from miclip.weights import synthetic_images
    g = golden(tag)
    R = MODEL_CONFIGS[name].image_resolution
    n = g["meta"]["n_images"]
    gold = synthetic_images(n, R, seed=g["meta"]["seed"])
    batch = synthetic_images(bs, R, seed=77)
    half = bs // 2
    rows = sorted({0, half - 1, half, bs - 1} | {3 + (bs // n) * i for i in range(n)})
    src = [i % n for i in range(len(rows))]
    batch[rows] = gold[src]
    _, m, _ = miclip.load(name, device="cuda", compute_dtype=dtype, surface="openai")
    m.set_splits(2)
    assert m.image_splits(bs) == splits, m.image_splits(bs)
    x = torch.from_numpy(batch).cuda()
    feats = m.encode_image(x).cpu()
    d = _one_minus_cos(feats[rows], g["image"][src])
    print(f"{name} {dtype} bs={bs} (splits {splits}): golden rows {rows} 1-cos max {d.max():.2e}")
    assert d.max() <= tol
    small = m.encode_image(torch.from_numpy(gold).cuda()).cpu()
    dc = centred_one_minus_cos(small, g["image"])
    print(f"{name} {dtype}: centred 1-cos over the {n} golden images {dc.max():.2e} (tol {ctol})")
    assert dc.max() <= ctol
    assert torch.equal(feats[rows], small[src]), \
        f"not batch invariant: max|d| {(feats[rows] - small[src]).abs().max().item():.3e}"
    # half-precision input in the compute dtype: bit-identical features
    hdt = torch.bfloat16 if dtype == "bf16" else torch.float16
    fh = m.encode_image(x.to(hdt)).cpu()
    assert torch.equal(fh, feats), f"{(fh != feats).any(1).sum().item()} rows differ"
    again = m.encode_image(x).cpu()
    assert torch.equal(again, feats), "large-batch encode is not deterministic"
    del m


def test_strong_split_shards_bitwise_vitl14():
    """SURVEY §8e's strong split: a global batch of 256 split G = 2/4/8/16 ways (128 /
    64 / 32 / 16 images per rank: M = 32 896 .. 4 112 GEMM rows, where the launcher
    switches to 192- / 128-row tiles and the 16-image parts to one stream) must encode each rank's
    slice to exactly the rows of the single-GPU bs=256 encode, so the sharded
    feature cache equals the single-GPU one bit for bit
    (aihab_utils/feature_cache.py:114-162; clip/model.py:216-235)."""
    import miclip
    from miclip.weights import synthetic_images
    _, m, _ = miclip.load("ViT-L/14", device="cuda", compute_dtype="fp16", surface="openai")
    x = torch.from_numpy(synthetic_images(256, 224, seed=5)).cuda()
    full = m.encode_image(x, normalize=True)
    for G in (2, 4, 8, 16):
        b = 256 // G
        for r in (0, G - 1):
            part = m.encode_image(x[r * b:(r + 1) * b], normalize=True)
            d = part != full[r * b:(r + 1) * b]
            assert not d.any(), f"G={G} rank {r}: {d.any(1).sum().item()} rows differ"
    del m
