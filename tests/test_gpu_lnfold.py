"""The folded LayerNorm (default fp16 path) and the benched configuration.

ln_1 / ln_2 (clip/model.py:151-157, applied at :184-185) are folded into the
QKV / c_fc GEMMs: LN(x) . W^T + b = (rstd / S) * (x . Wf^T - mean * colsum) + c
with Wf = W diag(gamma) * S (S a power of two, so W * gamma never rounds into the
fp16 subnormals), colsum = row sums of Wf, c = b + W beta (norm.hip ln_fold /
ln_stats, epilogue.h EpiStoreLN).

Op level: each piece against float64/fp32 torch, on LayerNorm parameters wider
than the random-init goldens (gamma log-uniform over [1e-3, 4] with random signs,
rows whose |mean| is 30-300x their std) and at the benched GEMM shapes (M = 257 *
{256, 128} and a ragged tail M), against the same GEMM fed the unfolded LayerNorm
output (the options={'ln_fold': False} path), with the same tolerance as tests/test_gpu_kernels.
Model level: fold vs ln_fold=False against the goldens, and ViT-L/14 fp16 at the
benched batch of 256 (2-stream split, persistent 256x256 GEMMs with row tails) with
the golden images placed across the split and the tail.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from miclip import _lib
    return _lib.load_library()


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(lib, rc):
    assert rc == 0, lib.miclip_last_error().decode()


def _ln_params(D, g):
    # |gamma| log-uniform in [1e-3, 4], random signs; beta ~ 0.5 N(0, 1)
    mag = torch.exp(torch.empty(D, device="cuda").uniform_(np.log(1e-3), np.log(4.0), generator=g))
    sign = torch.where(torch.rand(D, device="cuda", generator=g) < 0.2, -1.0, 1.0)
    return (mag * sign).contiguous(), (0.5 * torch.randn(D, device="cuda", generator=g)).contiguous()


def _stream_rows(M, D, g):
    """fp16 residual-stream rows: per-row offset mean 30-300x the row's spread,
    plus a few outlier channels like real CLIP residual streams."""
    spread = torch.exp(torch.empty(M, 1, device="cuda").uniform_(np.log(0.05), np.log(2.0), generator=g))
    mean = spread * torch.empty(M, 1, device="cuda").uniform_(30, 300, generator=g) * \
        torch.where(torch.rand(M, 1, device="cuda", generator=g) < 0.5, -1.0, 1.0)
    x = mean + spread * torch.randn(M, D, device="cuda", generator=g)
    x[:, 7] += 20 * spread[:, 0]
    return x.clamp(-60000, 60000).half()


def _fold(lib, W, gamma, beta, bias):
    N, K = W.shape
    Wf = torch.empty_like(W)
    cs = torch.empty(N, device="cuda")
    c = torch.empty(N, device="cuda")
    inv = torch.zeros(2, device="cuda")
    _check(lib, lib.miclip_op_ln_fold(0, W.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                      bias.data_ptr(), Wf.data_ptr(), cs.data_ptr(), c.data_ptr(),
                                      N, K, inv.data_ptr(), _stream()))
    return Wf, cs, c, inv


@pytest.mark.parametrize("R,D", [(7, 768), (513, 1024), (300, 1280), (65, 1536)])
def test_ln_stats(lib, R, D):
    g = torch.Generator(device="cuda").manual_seed(R + D)
    x = _stream_rows(R, D, g)
    st = torch.empty(R, 2, device="cuda")
    sc = torch.tensor([0.25, 0.0], device="cuda")
    st2 = torch.empty(R, 2, device="cuda")
    _check(lib, lib.miclip_op_ln_stats(x.data_ptr(), st.data_ptr(), R, D, None, _stream()))
    _check(lib, lib.miclip_op_ln_stats(x.data_ptr(), st2.data_ptr(), R, D, sc.data_ptr(), _stream()))
    torch.cuda.synchronize()
    xd = x.double()
    mu = xd.mean(1)
    rstd = 1 / torch.sqrt(((xd - mu[:, None]) ** 2).mean(1) + 1e-5)
    assert ((st[:, 0].double() - mu).abs() / mu.abs()).max().item() < 1e-6
    assert ((st[:, 1].double() - rstd) / rstd).abs().max().item() < 1e-4
    assert torch.equal(st2[:, 0], st[:, 0]) and torch.equal(st2[:, 1], st[:, 1] * 0.25)


@pytest.mark.parametrize("N,K", [(3072, 1024), (4096, 1024), (2304, 768), (512, 512)])
def test_ln_fold(lib, N, K):
    g = torch.Generator(device="cuda").manual_seed(N + K)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
    gamma, beta = _ln_params(K, g)
    bias = 0.02 * torch.randn(N, device="cuda", generator=g)
    Wf, cs, c, inv = _fold(lib, W, gamma, beta, bias)
    torch.cuda.synchronize()
    amax = (W.float() * gamma).abs().max().item()
    _, e = np.frexp(amax)
    S = 2.0 ** (15 - int(e))
    assert inv[0].item() == 1.0 / S
    # same fp32 expression, one RNE to fp16: bit for bit, and never subnormal
    ref = ((W.float() * gamma) * S).half()
    assert torch.equal(Wf, ref)
    # the scale's guarantee: every W*gamma within 2^28 of the largest stays a normal
    # fp16 (unscaled, |W gamma| < 6.1e-5 -- e.g. W ~ 0.03, gamma ~ 1e-3 -- would not)
    big = (W.float() * gamma).abs() >= amax * 2.0 ** -28
    assert (Wf.float().abs()[big] >= 2.0 ** -14).all(), "folded weights fell into the fp16 subnormals"
    assert Wf.float().abs().max().item() <= 2.0 ** 15
    cs_ref = Wf.double().sum(1)
    assert ((cs.double() - cs_ref).abs() <= 1e-6 * Wf.double().abs().sum(1)).all()
    c_ref = bias.double() + W.double() @ beta.double()
    assert ((c.double() - c_ref).abs() <= 1e-6 * (1 + (W.double().abs() @ beta.double().abs()))).all()


NO_TAIL = 1 << 16


@pytest.mark.parametrize("M", [65792, 32896, 16421])
@pytest.mark.parametrize("N", [3072, 4096])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_ln_vs_layernorm_linear(lib, M, N, act):
    """Folded GEMM vs fp32 F.layer_norm -> F.linear (-> QuickGELU), and vs the
    unfolded path (LayerNorm kernel -> fp16 h -> GEMM): the fold's error is
    within the tolerance the unfolded GEMM is held to, and comparable to it."""
    K = 1024
    g = torch.Generator(device="cuda").manual_seed(M + N + act)
    x = _stream_rows(M, K, g)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
    gamma, beta = _ln_params(K, g)
    bias = 0.02 * torch.randn(N, device="cuda", generator=g)
    Wf, cs, c, inv = _fold(lib, W, gamma, beta, bias)
    st = torch.empty(M, 2, device="cuda")
    _check(lib, lib.miclip_op_ln_stats(x.data_ptr(), st.data_ptr(), M, K, inv.data_ptr(), _stream()))
    out = torch.empty(M, N, device="cuda", dtype=torch.float16)
    _check(lib, lib.miclip_op_gemm_ln(0, x.data_ptr(), Wf.data_ptr(), c.data_ptr(), cs.data_ptr(),
                                      st.data_ptr(), out.data_ptr(), M, N, K, act, 0, _stream()))
    # unfolded: LayerNorm kernel (fp16 stream in, fp16 h out) -> GEMM store epilogue
    h = torch.empty(M, K, device="cuda", dtype=torch.float16)
    _check(lib, lib.miclip_op_layernorm(0, x.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                        h.data_ptr(), 2, M, K, _stream()))
    un = torch.empty(M, N, device="cuda", dtype=torch.float16)
    _check(lib, lib.miclip_op_gemm(0, h.data_ptr(), W.data_ptr(), bias.data_ptr(), un.data_ptr(),
                                   M, N, K, 0, act, 0, _stream()))
    torch.cuda.synchronize()
    err_f = err_u = 0.0
    amax = 0.0
    for r0 in range(0, M, 8192):          # fp32 reference in row chunks (memory)
        xs = x[r0:r0 + 8192].float()
        ref = torch.nn.functional.layer_norm(xs, (K,), gamma, beta, 1e-5) @ W.float().t() + bias
        if act:
            ref = ref * torch.sigmoid(1.702 * ref)
        amax = max(amax, ref.abs().max().item())
        err_f = max(err_f, (out[r0:r0 + 8192].float() - ref).abs().max().item())
        err_u = max(err_u, (un[r0:r0 + 8192].float() - ref).abs().max().item())
    tol = 4e-3 * max(1.0, amax)
    print(f"M={M} N={N} act={act}: max|ref| {amax:.2f}, fold err {err_f:.2e}, unfolded err {err_u:.2e}")
    assert err_f <= tol and err_u <= tol
    assert err_f <= 2 * err_u + 1e-3 * max(1.0, amax)


@pytest.mark.parametrize("M,N", [(16421, 3072), (16448, 4096), (4296, 4096)])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_ln_tail_bitexact(lib, M, N, act):
    """Row tail of the LN-epilogue GEMM (tail workgroups) equals the all-tile launch bit for bit."""
    K = 1024
    g = torch.Generator(device="cuda").manual_seed(M * 3 + N + act)
    x = _stream_rows(M, K, g)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
    gamma, beta = _ln_params(K, g)
    bias = 0.02 * torch.randn(N, device="cuda", generator=g)
    Wf, cs, c, inv = _fold(lib, W, gamma, beta, bias)
    st = torch.empty(M, 2, device="cuda")
    _check(lib, lib.miclip_op_ln_stats(x.data_ptr(), st.data_ptr(), M, K, inv.data_ptr(), _stream()))
    outs = []
    for v in (0, NO_TAIL | 259):
        o = torch.empty(M, N, device="cuda", dtype=torch.float16)
        _check(lib, lib.miclip_op_gemm_ln(0, x.data_ptr(), Wf.data_ptr(), c.data_ptr(), cs.data_ptr(),
                                          st.data_ptr(), o.data_ptr(), M, N, K, act, v, _stream()))
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "LN-epilogue tail rows differ from the all-tile launch"


def _one_minus_cos(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return (1 - torch.nn.functional.cosine_similarity(a, b, dim=-1)).numpy()


def test_fold_vs_unfolded_model(golden):
    """ViT-L/14 fp16: the default (folded) model and options={"ln_fold": False} both meet the
    tolerance against the reference goldens, image and text, and agree closely."""
    import miclip
    from miclip.weights import synthetic_images
    g = golden("vitl14")
    imgs = torch.from_numpy(synthetic_images(g["meta"]["n_images"], 224, seed=0)).cuda()
    tok = torch.from_numpy(g["tokens"]).long().cuda()
    res = {}
    for fold in ("1", "0"):
        _, m, _ = miclip.load("ViT-L/14", device="cuda", compute_dtype="fp16",
                              options={"ln_fold": fold == "1"})
        assert m.numerics()["lnfold"] == (fold == "1")
        res[fold] = (m.encode_image(imgs).cpu(), m.encode_text(tok)[1].cpu())
        del m
        torch.cuda.empty_cache()
    for fold, (fi, ft) in res.items():
        di, dt = _one_minus_cos(fi, g["image"]), _one_minus_cos(ft, g["text_proj"])
        print(f"fold={fold}: image 1-cos {di.max():.2e}, text 1-cos {dt.max():.2e}")
        assert di.max() <= COS_TOL and dt.max() <= COS_TOL
    assert _one_minus_cos(res["1"][0], res["0"][0]).max() <= 1e-4
    assert not torch.equal(res["1"][0], res["0"][0]), "ln_fold did not change the path"


def test_benched_config_vitl14_bs256(golden):
    """The benched configuration -- ViT-L/14 fp16, 256 images, default 2-stream split
    (M = 32896 rows per GEMM launch), persistent GEMMs with row tails, folded LN --
    with the 16 golden images spread over the batch (rows 0, 127, 128 and 255 among
    them: either side of the split and the last row): each within 1-cos 1e-3 of the
    reference, the centred features too, and bitwise equal to a 16-image encode of
    the same images (row order and batch invariance)."""
    import miclip
    from miclip.weights import synthetic_images
    from _parity import centred_one_minus_cos
    g = golden("vitl14")
    n = g["meta"]["n_images"]
    gold = synthetic_images(n, 224, seed=0)
    batch = synthetic_images(256, 224, seed=77)
    rows = [0, 127, 128, 255] + [r for r in range(3, 255, 16) if r not in (127, 128)][:n - 4]
    batch[rows] = gold
    _, m, _ = miclip.load("ViT-L/14", device="cuda", compute_dtype="fp16")
    m.set_splits(2)
    assert m.image_splits(256) == 2 and m.image_splits(n) == 1
    feats = m.encode_image(torch.from_numpy(batch).cuda()).cpu()
    d = _one_minus_cos(feats[rows], g["image"])
    dc = centred_one_minus_cos(feats[rows], g["image"])
    print(f"bs=256 golden rows 1-cos max {d.max():.2e}, centred {dc.max():.2e}")
    assert d.max() <= COS_TOL and dc.max() <= COS_TOL
    small = m.encode_image(torch.from_numpy(gold).cuda()).cpu()
    same = [torch.equal(feats[r], small[i]) for i, r in enumerate(rows)]
    print(f"bitwise equal to the {n}-image encode: {sum(same)}/{n}; max|d| "
          f"{(feats[rows] - small).abs().max().item():.3e}")
    assert all(same)
    again = m.encode_image(torch.from_numpy(batch).cuda()).cpu()
    assert torch.equal(feats, again), "bs=256 encode is not deterministic"
