"""The 4-wave persistent GEMM (gemm4s_kernel, op-level variants 508 / 516) against
the 8-wave default (variant 259) and fp32 torch.

gemm4s runs the same v_mfma_f32_16x16x32 chains in the same k order and calls the
epilogue functors' own value forms (val4 / val4ln / add_x), so every output
element must equal the 8-wave kernel's bit for bit -- tile rows, row-tail rows
(gemm_tail_wg on 4 waves) and the per-column / per-row epilogue operands
(bias, folded-LN column sums and row statistics) alike. Shapes: the ViT-L/14
bs=256 (M = 65 792) and half-batch (32 896) launches of every benched GEMM,
ragged M (tail tasks, narrow and wide), and small K. Reference: clip/model.py
:171-175 (in_proj, out_proj), :179-181 (c_fc, c_proj).
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {"fp16": (0, torch.float16), "bf16": (1, torch.bfloat16)}
VARIANTS = (508, 516)
BASE = 259


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from miclip import _lib
    return _lib.load_experiments()   # measured-slower kernel: diagnostic library only


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(lib, rc):
    assert rc == 0, lib.miclip_last_error().decode()


SHAPES = [(65792, 4096, 1024), (65792, 3072, 1024), (32896, 1024, 4096), (32896, 1024, 1024),
          (16421, 3072, 1024), (4352, 4096, 512), (4296, 4096, 256), (300, 256, 192),
          (16640, 3072, 256)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("epi,act,dt", [(0, 0, "fp16"), (0, 1, "fp16"), (0, 2, "fp16"),
                                        (4, 0, "fp16"), (0, 1, "bf16")])
def test_gemm4s_bitexact_vs_8wave(lib, M, N, K, epi, act, dt):
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + 7 * epi + act)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    X0 = (torch.randn(M, N, device="cuda", generator=g) * 2).half() if epi == 4 else None
    outs = {}
    for v in (BASE,) + VARIANTS:
        C = X0.clone() if epi == 4 else torch.empty(M, N, device="cuda", dtype=tdt)
        _check(lib, lib.miclip_op_gemm(code, A.data_ptr(), W.data_ptr(), bias.data_ptr(),
                                       C.data_ptr(), M, N, K, epi, act, v, _stream()))
        outs[v] = C
    torch.cuda.synchronize()
    for v in VARIANTS:
        d = (outs[v] != outs[BASE])
        assert not d.any(), (f"variant {v}: {d.any(1).sum().item()} rows differ from the 8-wave "
                             f"kernel (first {d.any(1).nonzero()[:4].flatten().tolist()})")
    # and against fp32 torch on a slice of rows (first, middle, tail)
    rows = torch.cat([torch.arange(0, 64), torch.arange(M // 2, M // 2 + 64),
                      torch.arange(max(0, M - 300), M)]).unique().cuda()
    ref = A[rows].float() @ W.float().t() + bias
    if act == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    elif act == 2:
        ref = torch.nn.functional.gelu(ref)
    if epi == 4:
        ref = X0[rows].float() + ref
    err = (outs[VARIANTS[0]][rows].float() - ref).abs().max().item()
    tol = (2e-2 if dt == "bf16" else 4e-3) * max(1.0, ref.abs().max().item())
    assert err <= tol, f"max|err| {err} > {tol}"


@pytest.mark.parametrize("M,N,K", [(65792, 4096, 1024), (65792, 3072, 1024), (16421, 3072, 1024),
                                   (4296, 4096, 256)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm4s_ln_epilogue_bitexact(lib, M, N, K, act):
    """Folded-LayerNorm epilogue (EpiStoreLN: per-row {mu, r}, per-column sums and
    folded bias, staged by LDS-DMA per tile) equals the 8-wave kernel bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(M + N + act)
    x = (torch.randn(M, K, device="cuda", generator=g) * 3 + 0.5).half()
    Wf = (torch.randn(N, K, device="cuda", generator=g) * 2 ** 14 * K ** -0.5).half()
    cs = torch.randn(N, device="cuda", generator=g) * 2 ** 10
    c = torch.randn(N, device="cuda", generator=g) * 0.05
    st = torch.stack([torch.randn(M, device="cuda", generator=g) * 0.1,
                      (torch.rand(M, device="cuda", generator=g) + 0.5) * 2 ** -14], 1).contiguous()
    outs = {}
    for v in (BASE,) + VARIANTS:
        o = torch.empty(M, N, device="cuda", dtype=torch.float16)
        _check(lib, lib.miclip_op_gemm_ln(0, x.data_ptr(), Wf.data_ptr(), c.data_ptr(), cs.data_ptr(),
                                          st.data_ptr(), o.data_ptr(), M, N, K, act, v, _stream()))
        outs[v] = o
    torch.cuda.synchronize()
    assert torch.isfinite(outs[BASE].float()).all()
    for v in VARIANTS:
        assert torch.equal(outs[v], outs[BASE]), f"variant {v} differs from the 8-wave kernel"


def test_gemm4s_rejects_unsupported(lib):
    """fp32 residual stream and M < 256 are refused by the explicit variant (no
    silent fallback)."""
    A = torch.zeros(128, 256, device="cuda", dtype=torch.float16)
    W = torch.zeros(256, 256, device="cuda", dtype=torch.float16)
    b = torch.zeros(256, device="cuda")
    C = torch.zeros(128, 256, device="cuda", dtype=torch.float16)
    assert lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), b.data_ptr(), C.data_ptr(),
                              128, 256, 256, 0, 0, 508, _stream()) != 0
    X = torch.zeros(300, 256, device="cuda")
    A2 = torch.zeros(300, 256, device="cuda", dtype=torch.float16)
    assert lib.miclip_op_gemm(0, A2.data_ptr(), W.data_ptr(), b.data_ptr(), X.data_ptr(),
                              300, 256, 256, 1, 0, 508, _stream()) != 0


@pytest.mark.parametrize("variant", [530, 531, 532, 533, 534])
@pytest.mark.parametrize("M,N,K,epi,act", [(65792, 4096, 1024, 0, 1), (32896, 1024, 4096, 4, 0),
                                           (16421, 1024, 1024, 4, 0)])
def test_gemm4s_dma_spread_variants_bitexact(lib, variant, M, N, K, epi, act):
    """The DMA-placement experiments change only when pieces are issued."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + variant)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    X0 = (torch.randn(M, N, device="cuda", generator=g) * 2).half() if epi == 4 else None
    outs = []
    for v in (BASE, variant):
        C = X0.clone() if epi == 4 else torch.empty(M, N, device="cuda", dtype=torch.float16)
        _check(lib, lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(),
                                       M, N, K, epi, act, v, _stream()))
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
