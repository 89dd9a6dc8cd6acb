"""The split-K GEMM of the CLS-only last vision block, at the op level
(miclip_op_gemm_splitk: gemm_nt_splitk_kernel + splitk_reduce_kernel).

The model reaches this path only from the last vision block's CLS rows
(capi.hip run_block cls_only; clip/model.py:226-229 keeps ln_post(x[:, 0, :])),
so until round 5 it was covered end to end only. Here, per epilogue (store with
each activation, the fp16 and fp32 residual streams, the folded-LN store):

  * integer operands (|a|, |w| <= 3, integer bias): every partial sum is an exact
    fp32 integer, so the split-K result must equal the unsplit GEMM's
    (miclip_op_gemm / miclip_op_gemm_ln, 128x128 kernel) BIT FOR BIT -- the
    reduce applies the same put4 epilogue to the same fp32 value -- and must not
    depend on sk;
  * fp16 operands: rows are batch-invariant (row r of an M = 257 launch equals row
    r of an M = 7 launch with the same sk; the model picks sk from K alone), and
    within the GEMM tolerance of fp32 torch;
at M in {1, 7, 257} (ragged 128-row tiles) and sk in {2, 4, 16}.
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


def _ptr(t):
    return None if t is None else t.data_ptr()


def _splitk(lib, code, A, W, bias, out, M, N, K, epi, act, sk, ln=None):
    ws = torch.empty(sk * M * N, device="cuda")
    c, colsum, stats = ln if ln is not None else (None, None, None)
    _check(lib, lib.miclip_op_gemm_splitk(code, A.data_ptr(), W.data_ptr(), _ptr(bias), _ptr(c),
                                          _ptr(colsum), _ptr(stats), out.data_ptr(), M, N, K, epi,
                                          act, sk, ws.data_ptr(), _stream()))


def _unsplit(lib, code, A, W, bias, out, M, N, K, epi, act, ln=None):
    if ln is None:
        _check(lib, lib.miclip_op_gemm(code, A.data_ptr(), W.data_ptr(), _ptr(bias), out.data_ptr(),
                                       M, N, K, epi, act, 128, _stream()))
    else:
        c, colsum, stats = ln
        _check(lib, lib.miclip_op_gemm_ln(code, A.data_ptr(), W.data_ptr(), c.data_ptr(),
                                          colsum.data_ptr(), stats.data_ptr(), out.data_ptr(), M, N,
                                          K, act, 128, _stream()))


def _operands(M, N, K, tdt, g, integer):
    if integer:
        A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(tdt)
        W = torch.randint(-3, 4, (N, K), device="cuda", generator=g).to(tdt)
        bias = torch.randint(-8, 9, (N,), device="cuda", generator=g).float()
    else:
        A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
        W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(tdt)
        bias = torch.randn(N, device="cuda", generator=g) * 0.1
    return A, W, bias


def _ln_operands(M, N, g):
    c = torch.randn(N, device="cuda", generator=g)
    colsum = torch.randn(N, device="cuda", generator=g) * 4
    stats = torch.stack([torch.randn(M, device="cuda", generator=g),
                         torch.rand(M, device="cuda", generator=g) * 0.01 + 1e-3], 1).contiguous()
    return c, colsum, stats


# (epi, act, output kind): 0 store (compute dtype), 1 fp32 residual, 4 fp16
# residual, 5 folded-LN store
CASES = [(0, 0), (0, 1), (0, 2), (1, 0), (4, 0), (5, 0), (5, 1)]


def _out(epi, M, N, tdt, g):
    if epi == 1:
        return torch.randint(-50, 51, (M, N), device="cuda", generator=g).float()
    if epi == 4:
        return torch.randint(-50, 51, (M, N), device="cuda", generator=g).half()
    return torch.full((M, N), 7.0, device="cuda", dtype=tdt)


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("epi,act", CASES)
@pytest.mark.parametrize("M", [1, 7, 257])
def test_splitk_integer_operands_bitexact(lib, dt, epi, act, M):
    code, tdt = DT[dt]
    N, K = 384, 1024
    g = torch.Generator(device="cuda").manual_seed(M * 31 + epi * 7 + act)
    A, W, bias = _operands(M, N, K, tdt, g, integer=True)
    ln = _ln_operands(M, N, g) if epi == 5 else None
    x0 = _out(epi, M, N, tdt, g)
    ref = x0.clone()
    _unsplit(lib, code, A, W, bias, ref, M, N, K, epi, act, ln)
    for sk in (2, 4, 16):
        out = x0.clone()
        _splitk(lib, code, A, W, bias, out, M, N, K, epi, act, sk, ln)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), f"sk={sk}: {(out != ref).sum().item()} elements differ"
    if epi in (0, 1, 4) and act == 0:
        # exact integers end to end: also equal to torch
        t = A.float() @ W.float().t() + bias
        want = {0: t.to(tdt), 1: x0 + t, 4: (x0.float() + t.half().float()).half()}[epi]
        assert torch.equal(ref, want)


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("epi,act", CASES)
def test_splitk_rows_batch_invariant(lib, dt, epi, act):
    code, tdt = DT[dt]
    N, K, sk = 256, 4096, 16
    g = torch.Generator(device="cuda").manual_seed(1000 + epi * 7 + act)
    A, W, bias = _operands(257, N, K, tdt, g, integer=False)
    ln = _ln_operands(257, N, g) if epi == 5 else None
    x0 = _out(epi, 257, N, tdt, g)
    big = x0.clone()
    _splitk(lib, code, A, W, bias, big, 257, N, K, epi, act, sk, ln)
    small = x0[:7].clone()
    ln7 = None if ln is None else (ln[0], ln[1], ln[2][:7].contiguous())
    _splitk(lib, code, A[:7].contiguous(), W, bias, small, 7, N, K, epi, act, sk, ln7)
    torch.cuda.synchronize()
    assert torch.equal(big[:7], small)
    if epi in (0, 1, 4) and act == 0:
        t = A.float() @ W.float().t() + bias
        want = {0: t, 1: x0 + t, 4: x0.float() + t}[epi]
        tol = 4e-3 * want.abs().max().item() + (0.06 if epi == 4 else 0.0)
        assert (big.float() - want).abs().max().item() <= tol


def test_splitk_refuses_bad_shapes(lib):
    z = torch.zeros(1 << 16, device="cuda")
    ws = torch.zeros(1 << 16, device="cuda")
    p = z.data_ptr()
    # K not a multiple of 64 * sk, sk out of range, missing folded-LN operands
    assert lib.miclip_op_gemm_splitk(0, p, p, p, None, None, None, p, 7, 128, 192, 0, 0, 4,
                                     ws.data_ptr(), _stream()) != 0
    assert lib.miclip_op_gemm_splitk(0, p, p, p, None, None, None, p, 7, 128, 1024, 0, 0, 1,
                                     ws.data_ptr(), _stream()) != 0
    assert lib.miclip_op_gemm_splitk(0, p, p, p, None, None, None, p, 7, 128, 1024, 5, 0, 4,
                                     ws.data_ptr(), _stream()) != 0
