"""The persistent MX-fp8 GEMM (gemm256s_mx_kernel, miclip_op_gemm_mx_v variant 2, the
default where K >= 256) against the one-tile-per-workgroup kernel (variant 1).

Both run the same scaled-MFMA chains in the same k order and the same epilogue
arithmetic, so every output byte -- fp16 stores, the fp16 residual stream, MX-fp8
data and its scale plane -- must be identical: full-size ViT-H/14 launches (bs=256
per stream: 65 792 rows), ragged row counts (partial last tiles, the persistent
kernel's tile loop ending on a partial round) and the smallest K it takes. The
numerics of the kernel itself are pinned by test_gpu_mx.py (dequantised-operand
products, epilogue within one e4m3 step of the oracle). Reference shapes:
clip/model.py:171-181 at open_clip ViT-H/14 widths.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


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


def _mx(lib, x):
    """fp16 rows -> MX-fp8 data + scale plane on the GPU (quant_mx)."""
    R, K = x.shape
    q = torch.empty(R, K, dtype=torch.uint8, device="cuda")
    s = torch.zeros(int(lib.miclip_mx_scale_bytes(R, K)), dtype=torch.uint8, device="cuda")
    _check(lib, lib.miclip_op_quant_mx(x.data_ptr(), 1, R, K, q.data_ptr(), s.data_ptr(), _stream()))
    return q, s


def _run(lib, qa, sa, qw, sw, bias, M, N, K, epi, act, variant, X0=None):
    if epi == 5:
        C = torch.empty(M, N, dtype=torch.uint8, device="cuda")
        CS = torch.zeros(int(lib.miclip_mx_scale_bytes(M, N)), dtype=torch.uint8, device="cuda")
    else:
        C = X0.clone() if epi == 1 else torch.empty(M, N, dtype=torch.float16, device="cuda")
        CS = None
    _check(lib, lib.miclip_op_gemm_mx_v(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(),
                                        bias.data_ptr(), C.data_ptr(),
                                        CS.data_ptr() if CS is not None else None, M, N, K, epi,
                                        act, variant, _stream()))
    return C, CS


SHAPES = [(65792, 3840, 1280, 0, 0), (65792, 1280, 1280, 1, 0), (65792, 5120, 1280, 5, 3),
          (65792, 1280, 5120, 1, 0), (16421, 3840, 1280, 0, 0), (16421, 5120, 1280, 5, 2),
          (4296, 5120, 512, 5, 1), (300, 1280, 256, 1, 0), (300, 256, 256, 0, 1),
          (257, 512, 512, 5, 0), (1000, 768, 1280, 0, 2)]


@pytest.mark.parametrize("M,N,K,epi,act", SHAPES)
def test_persistent_mx_bitexact(lib, M, N, K, epi, act):
    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + K + epi + act)
    A = (torch.randn(M, K, device="cuda", generator=g) * 2).half()
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    X0 = (torch.randn(M, N, device="cuda", generator=g) * 3).half() if epi == 1 else None
    qa, sa = _mx(lib, A)
    qw, sw = _mx(lib, W)
    c1, s1 = _run(lib, qa, sa, qw, sw, bias, M, N, K, epi, act, 1, X0)
    c2, s2 = _run(lib, qa, sa, qw, sw, bias, M, N, K, epi, act, 2, X0)
    c0, _ = _run(lib, qa, sa, qw, sw, bias, M, N, K, epi, act, 0, X0)
    torch.cuda.synchronize()
    if epi != 5:
        assert torch.isfinite(c1.float()).all()
    d = c1 != c2
    assert not d.any(), (f"{d.any(1).sum().item()} rows differ "
                         f"(first {d.any(1).nonzero()[:4].flatten().tolist()})")
    assert torch.equal(c0, c2)           # the default launch is the persistent kernel
    if epi == 5:
        assert torch.equal(s1, s2)
        assert int(s1.max()) > 0          # scales were written


def test_persistent_mx_refusals(lib):
    """variant 2 needs K >= 256 (refused, not silently replaced); variant 0 at K =
    128 runs the one-tile kernel; unknown variants are refused."""
    M, N, K = 512, 256, 128
    # operands quantised at K = 256 (quant_mx's minimum) and read as K = 128 rows:
    # in bounds, and the same bytes for both kernels
    A = torch.randn(M, 256, device="cuda").half()
    W = torch.randn(N, 256, device="cuda").half()
    bias = torch.zeros(N, device="cuda")
    qa, sa = _mx(lib, A)
    qw, sw = _mx(lib, W)
    C = torch.empty(M, N, dtype=torch.float16, device="cuda")
    args = (qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
            C.data_ptr(), None, M, N, K, 0, 0)
    assert lib.miclip_op_gemm_mx_v(*args, 2, _stream()) != 0
    assert lib.miclip_op_gemm_mx_v(*args, 3, _stream()) != 0
    _check(lib, lib.miclip_op_gemm_mx_v(*args, 0, _stream()))
    c0 = C.clone()
    _check(lib, lib.miclip_op_gemm_mx_v(*args, 1, _stream()))
    torch.cuda.synchronize()
    assert torch.equal(c0, C)
