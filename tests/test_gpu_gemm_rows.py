"""192- and 128-row tiles of the persistent GEMM (gemm256s_kernel RB = 3 / 2, op-level
variants 192, 129 = 128-row tiles, 130 = 128-row tiles + row tail; the launcher's
choices where 256-row tiles leave CUs idle, e.g. the ViT-B/32 bs=256 out-projection /
c_proj at M = 12 800, N = 768, or ViT-L/14 at 16-64 images per GPU, SURVEY §8e's strong
split) against the 256-row default (variant 259), and the by-size launcher (variant 0).

Same MFMA chains in the same k order and the same epilogue functors, so every output
element must be identical -- for the fp16 store (with QuickGELU / GELU), the folded-
LayerNorm store and the fp16 residual stream, fp16 and bf16 operands, partial last
tiles and full ones. Reference: clip/model.py:171-181 (the block's projections).
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {"fp16": (0, torch.float16), "bf16": (1, torch.bfloat16)}


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


SHAPES = [(12800, 768, 768), (12800, 768, 3072), (12800, 2304, 768), (12800, 3072, 768),
          (6400, 768, 768), (1000, 1024, 512), (192, 256, 128), (383, 512, 256), (65792, 1024, 1024),
          # ViT-L/14 per-rank shapes of the strong split: 32 / 16 / 64 images
          (8224, 1024, 1024), (8224, 1024, 4096), (8224, 3072, 1024), (4112, 4096, 1024),
          (16448, 1024, 1024)]
VARIANTS = (192, 129, 130, 0)


@pytest.mark.parametrize("v", VARIANTS)
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("epi,act,dt", [(0, 0, "fp16"), (0, 1, "fp16"), (0, 2, "bf16"),
                                        (4, 0, "fp16"), (4, 0, "bf16")])
def test_gemm_rows_bitexact_vs_256(lib, v, M, N, K, epi, act, dt):
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + 7 * epi + act + code)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    X0 = (torch.randn(M, N, device="cuda", generator=g) * 2).half() if epi == 4 else None
    outs = {}
    for vv in (259, v):
        C = X0.clone() if epi == 4 else torch.empty(M, N, device="cuda", dtype=tdt)
        _check(lib, lib.miclip_op_gemm(code, A.data_ptr(), W.data_ptr(), bias.data_ptr(),
                                       C.data_ptr(), M, N, K, epi, act, vv, _stream()))
        outs[vv] = C
    torch.cuda.synchronize()
    d = outs[v] != outs[259]
    assert not d.any(), (f"{d.any(1).sum().item()} rows differ "
                         f"(first {d.any(1).nonzero()[:4].flatten().tolist()})")
    rows = torch.cat([torch.arange(0, 64), torch.arange(max(0, M - 200), M)]).unique().cuda()
    ref = A[rows].float() @ W.float().t() + bias
    if act == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    elif act == 2:
        ref = torch.nn.functional.gelu(ref)
    if epi == 4:
        ref = X0[rows].float() + ref
    err = (outs[v][rows].float() - ref).abs().max().item()
    tol = (2e-2 if dt == "bf16" else 4e-3) * max(1.0, ref.abs().max().item())
    assert err <= tol, f"max|err| {err} > {tol}"


@pytest.mark.parametrize("v", VARIANTS)
@pytest.mark.parametrize("M,N,K", [(12800, 2304, 768), (12800, 3072, 768), (1000, 1024, 512),
                                   (8224, 3072, 1024), (4112, 4096, 1024), (16448, 3072, 1024)])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_rows_ln_epilogue_bitexact(lib, v, M, N, K, act):
    """Folded-LayerNorm epilogue (row statistics of 192 / 128 rows DMA'd per tile)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + act)
    x = (torch.randn(M, K, device="cuda", generator=g) * 3 + 0.5).half()
    Wf = (torch.randn(N, K, device="cuda", generator=g) * 2 ** 14 * K ** -0.5).half()
    cs = torch.randn(N, device="cuda", generator=g) * 2 ** 10
    c = torch.randn(N, device="cuda", generator=g) * 0.05
    st = torch.stack([torch.randn(M, device="cuda", generator=g) * 0.1,
                      (torch.rand(M, device="cuda", generator=g) + 0.5) * 2 ** -14], 1).contiguous()
    outs = {}
    for vv in (259, v):
        o = torch.empty(M, N, device="cuda", dtype=torch.float16)
        _check(lib, lib.miclip_op_gemm_ln(0, x.data_ptr(), Wf.data_ptr(), c.data_ptr(), cs.data_ptr(),
                                          st.data_ptr(), o.data_ptr(), M, N, K, act, vv, _stream()))
        outs[vv] = o
    torch.cuda.synchronize()
    assert torch.isfinite(outs[259].float()).all()
    assert torch.equal(outs[v], outs[259])


@pytest.mark.parametrize("v", [192, 129, 130])
def test_gemm_rows_refused_for_row_staged_epilogues(lib, v):
    """Variants 192 / 129 / 130 need a transposed-accumulator epilogue: the fp32
    residual stream is refused, not silently run on 256-row tiles."""
    A = torch.zeros(300, 256, device="cuda", dtype=torch.float16)
    W = torch.zeros(256, 256, device="cuda", dtype=torch.float16)
    b = torch.zeros(256, device="cuda")
    X = torch.zeros(300, 256, device="cuda")
    assert lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), b.data_ptr(), X.data_ptr(),
                              300, 256, 256, 1, 0, v, _stream()) != 0
