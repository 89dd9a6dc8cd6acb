"""Ping-pong persistent GEMM (gemm.hip gemm_pp_kernel, variants 400-419).

Two 4-wave workgroups per CU on 256x128 tiles, 32-k steps through a 3-slot LDS
ring, register epilogue with v_permlane16_swap 16-B row pieces. It runs the
same v_mfma_f32_16x16x32 chain in the same k order as every other GEMM path,
so its outputs must equal the default kernel's BIT FOR BIT (batch invariance
of the encode relies on it), on full tiles, on a partial last tile-row (rows
past M read through the buffer descriptor's range check, never stored) and
for every epilogue the fp16 model runs: plain (QKV), QuickGELU (c_fc), exact
GELU (open_clip c_fc), fp16 residual (out-proj, c_proj) and the folded
LayerNorm (QKV / c_fc with ln_1 / ln_2 folded). Repeated launches must agree
(a missing wait or barrier shows up as run-to-run differences).
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

PP = 400          # variant 400 + d: second workgroup per CU starts d us late


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


SHAPES = [(16448, 1024, 1024), (16421, 3072, 256), (4112, 4096, 512), (1000, 256, 128),
          (32896, 4096, 1024), (300, 1024, 4096)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("epi,act,dt", [(0, 0, 0), (0, 1, 0), (0, 2, 0), (4, 0, 0), (0, 1, 1)])
@pytest.mark.parametrize("delay", [0, 4])
def test_pp_bitexact_vs_default(lib, M, N, K, epi, act, dt, delay):
    tdt = torch.float16 if dt == 0 else torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(M + N + K + epi + act)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    X0 = (torch.randn(M, N, device="cuda", generator=g)).to(tdt) if epi == 4 else None
    outs = []
    for v in (0, PP + delay, PP + delay, PP + delay):
        C = X0.clone() if epi == 4 else torch.full((M, N), 7.0, device="cuda", dtype=tdt)
        _check(lib, lib.miclip_op_gemm(dt, A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(),
                                       M, N, K, epi, act, v, _stream()))
        outs.append(C)
    torch.cuda.synchronize()
    for i, o in enumerate(outs[1:]):
        nd = (o != outs[0]).sum().item()
        assert nd == 0, f"run {i}: {nd} elements differ from the default kernel"
    # and within the GEMM tolerance of fp32 on the last rows (the partial tile)
    ref = A[-200:].float() @ W.float().t() + bias
    if act == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    if act == 2:
        ref = torch.nn.functional.gelu(ref)
    if epi == 4:
        ref = X0[-200:].float() + ref
    err = (outs[1][-200:].float() - ref).abs().max().item()
    assert err <= (2e-2 if dt else 4e-3) * max(1.0, ref.abs().max().item()), err


def _fold(lib, W, gamma, beta, bias):
    N, K = W.shape
    Wf = torch.empty_like(W)
    cs = torch.empty(N, device="cuda")
    c = torch.empty(N, device="cuda")
    inv = torch.zeros(2, device="cuda")
    _check(lib, lib.miclip_op_ln_fold(0, W.data_ptr(), gamma.data_ptr(), beta.data_ptr(), bias.data_ptr(),
                                      Wf.data_ptr(), cs.data_ptr(), c.data_ptr(), N, K, inv.data_ptr(),
                                      _stream()))
    return Wf, cs, c, inv


@pytest.mark.parametrize("M,N", [(32896, 4096), (16421, 3072), (2056, 1024)])
@pytest.mark.parametrize("act", [0, 1])
def test_pp_ln_bitexact_vs_default(lib, M, N, act):
    K = 1024
    g = torch.Generator(device="cuda").manual_seed(M + N + act)
    x = (torch.randn(M, K, device="cuda", generator=g) * 2 + 0.5).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
    gamma = torch.rand(K, device="cuda", generator=g) + 0.5
    beta = 0.1 * torch.randn(K, device="cuda", generator=g)
    bias = 0.02 * torch.randn(N, device="cuda", generator=g)
    Wf, cs, c, inv = _fold(lib, W, gamma, beta, bias)
    st = torch.empty(M, 2, device="cuda")
    _check(lib, lib.miclip_op_ln_stats(x.data_ptr(), st.data_ptr(), M, K, inv.data_ptr(), _stream()))
    outs = []
    for v in (0, PP, PP + 4):
        o = torch.full((M, N), 7.0, device="cuda", dtype=torch.float16)
        _check(lib, lib.miclip_op_gemm_ln(0, x.data_ptr(), Wf.data_ptr(), c.data_ptr(), cs.data_ptr(),
                                          st.data_ptr(), o.data_ptr(), M, N, K, act, v, _stream()))
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), f"{(o != outs[0]).sum().item()} elements differ"


def test_pp_rejects_unsupported(lib):
    A = torch.zeros(256, 96, device="cuda", dtype=torch.float16)
    W = torch.zeros(128, 96, device="cuda", dtype=torch.float16)
    b = torch.zeros(128, device="cuda")
    C = torch.zeros(256, 128, device="cuda", dtype=torch.float16)
    # K must be a multiple of 64 and at least 128
    assert lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), b.data_ptr(), C.data_ptr(), 256, 128, 96,
                              0, 0, PP, _stream()) != 0
