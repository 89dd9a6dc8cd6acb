"""Kernel-level parity of the HIP path (through the C ABI) against torch fp32.

Each test feeds the same rounded (fp16/bf16) operands to the kernel and to a
plain fp32 torch reference of the same op, and bounds the difference.
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


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("M,N,K,variant", [(300, 256, 192, 0), (128, 128, 64, 0), (65, 384, 1024, 0),
                                          (1000, 768, 3072, 128), (1000, 768, 3072, 256),
                                          (300, 256, 192, 256), (257, 512, 64, 256),
                                          (4096, 1024, 1024, 0), (33, 2304, 768, 256),
                                          (33, 2304, 768, 257), (600, 1024, 4096, 257),
                                          (1000, 768, 3072, 3), (300, 256, 192, 3), (257, 512, 64, 3),
                                          (65792, 1024, 128, 3), (2000, 2304, 256, 3),
                                          (65792, 1024, 1024, 3), (700, 2048, 320, 3),
                                          (1000, 768, 3072, 258), (300, 256, 192, 258), (257, 512, 64, 258),
                                          (4096, 1024, 1024, 258), (33, 2304, 128, 258),
                                          (1000, 768, 3072, 260), (300, 256, 192, 260), (257, 512, 64, 260),
                                          (4096, 1024, 1024, 260), (33, 2304, 128, 260),
                                          (1000, 768, 3072, 259), (300, 256, 192, 259), (257, 512, 64, 259),
                                          (4096, 1024, 1024, 259), (33, 2304, 128, 259),
                                          (65792, 1024, 1024, 259), (16448, 3072, 256, 259)])
@pytest.mark.parametrize("epi,act", [(0, 0), (0, 1), (0, 2), (1, 0), (2, 0), (4, 0)])
def test_gemm(lib, dt, M, N, K, variant, epi, act):
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + epi * 3 + act)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    ref = A.float() @ W.float().t() + bias
    if epi == 0:
        if act == 1:
            ref = ref * torch.sigmoid(1.702 * ref)
        elif act == 2:
            ref = torch.nn.functional.gelu(ref)
        C = torch.empty(M, N, device="cuda", dtype=tdt)
    elif epi == 1:
        X0 = torch.randn(M, N, device="cuda", generator=g)
        C = X0.clone()
        ref = X0 + ref
    elif epi == 4:   # fp16 residual stream (fp16 or bf16 operands)
        if dt != "fp16" and variant in (2, 300):
            return   # the experiments' kernels are checked on fp16 only
        X0 = torch.randn(M, N, device="cuda", generator=g).half()
        C = X0.clone()
        ref = X0.float() + ref
    else:
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    _check(lib, lib.miclip_op_gemm(code, A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(),
                                   M, N, K, epi, act, variant, _stream()))
    torch.cuda.synchronize()
    err = (C.float() - ref).abs().max().item()
    tol = ((2e-2 if dt == "bf16" else 4e-3) * max(1.0, ref.abs().max().item()) if epi in (0, 4)
           else 2e-4 * K ** 0.5)
    assert err <= tol, f"max|err| {err} > {tol}"


NO_TAIL = 1 << 16   # gemm.hip kGemmNoTail: every row in 256x256 tiles


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("M,N,K", [(16448, 1024, 1024), (16421, 1024, 256), (4112, 4096, 512),
                                   (16448, 3072, 256), (16500, 1024, 2048), (4352, 4096, 512),
                                   (4296, 4096, 256), (16640, 3072, 256)])
@pytest.mark.parametrize("variant", [258, 260, 256, 258 | (1 << 17), 260 | (1 << 17), 259])
@pytest.mark.parametrize("epi,act", [(0, 0), (0, 1), (0, 2), (1, 0), (2, 0), (4, 0)])
def test_gemm_tail_bitexact(lib, dt, M, N, K, variant, epi, act):
    """Row tail of a 256x256 launch (rows past the last whole round of tiles,
    computed as 16-row slivers of tiles (SCHED 2) or by tail workgroups) equals the all-tile launch bit for bit
    and the fp32 reference within the GEMM tolerance."""
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(M + N + K + epi + act)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    if epi == 0:
        mk = lambda: torch.empty(M, N, device="cuda", dtype=tdt)  # noqa: E731
    elif epi == 1:
        X0 = torch.randn(M, N, device="cuda", generator=g)
        mk = X0.clone
    elif epi == 4:   # fp16 residual stream (fp16 or bf16 operands)
        X0 = torch.randn(M, N, device="cuda", generator=g).half()
        mk = X0.clone
    else:
        mk = lambda: torch.empty(M, N, device="cuda", dtype=torch.float32)  # noqa: E731
    outs = []
    for v in (variant, variant | NO_TAIL):
        C = mk()
        _check(lib, lib.miclip_op_gemm(code, A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(),
                                       M, N, K, epi, act, v, _stream()))
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "tail rows differ from the all-tile launch"
    ref = A[-300:].float() @ W.float().t() + bias
    if epi == 0 and act == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    if epi == 0 and act == 2:
        ref = torch.nn.functional.gelu(ref)
    if epi in (1, 4):
        ref = X0[-300:].float() + ref
    err = (outs[0][-300:].float() - ref).abs().max().item()
    tol = ((2e-2 if dt == "bf16" else 4e-3) * max(1.0, ref.abs().max().item()) if epi in (0, 4)
           else 2e-4 * K ** 0.5)
    assert err <= tol, f"max|err| {err} > {tol}"


def test_gemm_rejects_bad_shapes(lib):
    A = torch.zeros(16, 64, device="cuda", dtype=torch.float16)
    W = torch.zeros(100, 64, device="cuda", dtype=torch.float16)
    C = torch.zeros(16, 100, device="cuda", dtype=torch.float16)
    rc = lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), None, C.data_ptr(), 16, 100, 64, 0, 0, 0, _stream())
    assert rc == -1
    # 256 tile needs N % 256 == 0
    W2 = torch.zeros(384, 64, device="cuda", dtype=torch.float16)
    C2 = torch.zeros(16, 384, device="cuda", dtype=torch.float16)
    assert lib.miclip_op_gemm(0, A.data_ptr(), W2.data_ptr(), None, C2.data_ptr(), 16, 384, 64, 0, 0, 256, _stream()) == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("R,D", [(7, 768), (513, 1024), (64, 512), (3, 1280)])
def test_layernorm(lib, dt, R, D):
    code, tdt = DT[dt]
    x = torch.randn(R, D, device="cuda") * 3 + 0.5
    gam = 1 + 0.1 * torch.randn(D, device="cuda")
    bet = 0.05 * torch.randn(D, device="cuda")
    ref = torch.nn.functional.layer_norm(x, (D,), gam, bet, 1e-5)
    out32 = torch.empty(R, D, device="cuda")
    _check(lib, lib.miclip_op_layernorm(code, x.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        out32.data_ptr(), 1, R, D, _stream()))
    outt = torch.empty(R, D, device="cuda", dtype=tdt)
    _check(lib, lib.miclip_op_layernorm(code, x.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        outt.data_ptr(), 0, R, D, _stream()))
    torch.cuda.synchronize()
    assert (out32 - ref).abs().max().item() < 1e-4
    assert (outt.float() - ref).abs().max().item() < (3e-2 if dt == "bf16" else 4e-3)


@pytest.mark.parametrize("D", [1024, 1280])
def test_layernorm_row_paths_bitexact(lib, D):
    """fp16-stream LayerNorm launches of >= 1024 x 32 rows take 32-row workgroups (each wave
    4 row pairs), smaller ones 8-row workgroups: the same per-row arithmetic, so a row's
    output is identical whichever path ran it -- fp16 out, fp16 in place, and (D = 1280)
    MX-fp8 rows and scales. R odd: the last pair's second row is past the end."""
    R = 33001
    g = torch.Generator(device="cuda").manual_seed(D)
    x = ((torch.randn(R, D, device="cuda", generator=g) * 3 + 0.5)).half()
    gam = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    bet = 0.05 * torch.randn(D, device="cuda", generator=g)
    full = torch.empty(R, D, device="cuda", dtype=torch.float16)
    _check(lib, lib.miclip_op_layernorm(0, x.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        full.data_ptr(), 2, R, D, _stream()))
    xin = x.clone()
    _check(lib, lib.miclip_op_layernorm(0, xin.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        xin.data_ptr(), 2, R, D, _stream()))
    lo, hi = (0, 1024), (R - 233, R)
    parts = []
    for a, b in (lo, hi):
        o = torch.empty(b - a, D, device="cuda", dtype=torch.float16)
        _check(lib, lib.miclip_op_layernorm(0, x[a:b].data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                            o.data_ptr(), 2, b - a, D, _stream()))
        parts.append(o)
    torch.cuda.synchronize()
    assert torch.equal(xin, full)
    assert torch.equal(parts[0], full[:1024]) and torch.equal(parts[1], full[R - 233:])
    ref = torch.nn.functional.layer_norm(x.float(), (D,), gam, bet, 1e-5)
    assert (full.float() - ref).abs().max().item() < 4e-3
    if D == 1280:   # MX rows: D a multiple of 128
        sb = int(lib.miclip_mx_scale_bytes(R, D))
        q = torch.empty(R, D, dtype=torch.uint8, device="cuda")
        sc = torch.zeros(sb, dtype=torch.uint8, device="cuda")
        _check(lib, lib.miclip_op_layernorm_mx(x.data_ptr(), 1, gam.data_ptr(), bet.data_ptr(),
                                               q.data_ptr(), sc.data_ptr(), R, D, _stream()))
        blk = (D // 128) * 1024            # scale bytes per 256-row block
        for a, b in ((0, 1024), (32768, R)):   # slices start on a 256-row block
            qa = torch.empty(b - a, D, dtype=torch.uint8, device="cuda")
            sa = torch.zeros(int(lib.miclip_mx_scale_bytes(b - a, D)), dtype=torch.uint8, device="cuda")
            _check(lib, lib.miclip_op_layernorm_mx(x[a:b].data_ptr(), 1, gam.data_ptr(), bet.data_ptr(),
                                                   qa.data_ptr(), sa.data_ptr(), b - a, D, _stream()))
            torch.cuda.synchronize()
            assert torch.equal(qa, q[a:b])
            nb = (b - a + 255) // 256
            assert torch.equal(sa[:nb * blk], sc[a // 256 * blk:(a // 256 + nb) * blk])


@pytest.mark.parametrize("R,D", [(7, 768), (513, 1024), (3, 1280), (300, 1536)])
def test_layernorm_fp16_stream(lib, R, D):
    """fp16 input (the fp16 residual stream): fp32 out, fp16 out, and fp16 in place (ln_pre)."""
    x = (torch.randn(R, D, device="cuda") * 3 + 0.5).half()
    gam = 1 + 0.1 * torch.randn(D, device="cuda")
    bet = 0.05 * torch.randn(D, device="cuda")
    ref = torch.nn.functional.layer_norm(x.float(), (D,), gam, bet, 1e-5)
    out32 = torch.empty(R, D, device="cuda")
    _check(lib, lib.miclip_op_layernorm(0, x.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        out32.data_ptr(), 1 | 2, R, D, _stream()))
    out16 = torch.empty(R, D, device="cuda", dtype=torch.float16)
    _check(lib, lib.miclip_op_layernorm(0, x.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        out16.data_ptr(), 2, R, D, _stream()))
    xin = x.clone()
    _check(lib, lib.miclip_op_layernorm(0, xin.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        xin.data_ptr(), 2, R, D, _stream()))
    torch.cuda.synchronize()
    assert (out32 - ref).abs().max().item() < 1e-4
    assert (out16.float() - ref).abs().max().item() < 4e-3
    assert torch.equal(xin, out16)
    # bf16 compute on the fp16 stream: bf16 out (same statistics, rounded to bf16)
    outb = torch.empty(R, D, device="cuda", dtype=torch.bfloat16)
    _check(lib, lib.miclip_op_layernorm(1, x.data_ptr(), gam.data_ptr(), bet.data_ptr(),
                                        outb.data_ptr(), 2, R, D, _stream()))
    torch.cuda.synchronize()
    assert (outb.float() - ref).abs().max().item() < 3e-2
    assert torch.equal(outb, out32.to(torch.bfloat16)) or \
        (outb.float() - out32.to(torch.bfloat16).float()).abs().max().item() <= 2 ** -6 * ref.abs().max().item()


def _attn_ref(qkv, B, N, H, causal, dh=64):
    q, k, v = qkv.float().view(B, N, 3, H, dh).permute(2, 0, 3, 1, 4)
    mask = None
    if causal:
        mask = torch.full((N, N), float("-inf"), device=qkv.device).triu_(1)
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=mask)
    return o.permute(0, 2, 1, 3).reshape(B * N, H * dh)


@pytest.mark.parametrize("variant", [1, 2, 4])
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("B,N,H,causal", [(2, 50, 3, 0), (3, 77, 2, 1), (2, 257, 2, 0),
                                          (1, 577, 2, 0), (2, 197, 1, 0), (1, 32, 1, 1),
                                          (1, 1, 1, 0), (2, 100, 2, 1), (37, 257, 16, 0),
                                          (5, 77, 12, 1)])
def test_attention(lib, dt, B, N, H, causal, variant):
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N + H + causal)
    qkv = (torch.randn(B * N, 3 * H * 64, device="cuda", generator=g) * 1.5).to(tdt)
    out = torch.empty(B * N, H * 64, device="cuda", dtype=tdt)
    _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), B, N, H, 64, causal,
                                        variant, _stream()))
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, B, N, H, causal)
    err = (out.float() - ref).abs().max().item()
    assert err < (4e-2 if dt == "bf16" else 6e-3), err


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("B,N,H", [(2, 257, 2), (37, 257, 16), (3, 256, 3), (2, 259, 2), (5, 258, 4),
                                   (1, 257, 1)])
def test_attention_x8(lib, dt, B, N, H):
    """Two-workgroups-per-CU kernel (variant 8; default at N = 257): 8 full query
    chunks + a ragged chunk split over the waves' key ranges and merged."""
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N + H + 8)
    qkv = (torch.randn(B * N, 3 * H * 64, device="cuda", generator=g) * 1.5).to(tdt)
    out = torch.empty(B * N, H * 64, device="cuda", dtype=tdt)
    for variant in (8, 0):
        out.fill_(7.0)
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), B, N, H, 64, 0,
                                            variant, _stream()))
        torch.cuda.synchronize()
        ref = _attn_ref(qkv, B, N, H, 0)
        err = (out.float() - ref).abs().max().item()
        assert err < (4e-2 if dt == "bf16" else 6e-3), (variant, err)
    # outside 256 <= N <= 259 (or causal) variant 8 is refused, not silently run
    for n, causal in ((200, 0), (260, 0), (287, 0), (257, 1)):
        assert lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), 1, n, H, 64, causal, 8,
                                       _stream()) != 0


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("N", [257, 258, 259])
def test_attention_x8_many_heads_per_workgroup(lib, dt, N):
    """Variant 8 walks hpw > 1 heads per workgroup at the benched batch (2048
    heads over 2 x 256 slots). The ragged queries' extra keys must be taken
    before the closing barrier: after it other waves DMA the next head into the
    same K/V image. Each head's arithmetic does not depend on hpw, so the whole
    batch must equal, bit for bit, launches of 16 images (256 heads: hpw = 1),
    on every one of several repeats (a race would vary run to run)."""
    code, tdt = DT[dt]
    B, H = 160, 16                     # 2560 heads: hpw = 5 on 256 CUs
    g = torch.Generator(device="cuda").manual_seed(N + 31)
    qkv = (torch.randn(B * N, 3 * H * 64, device="cuda", generator=g) * 1.5).to(tdt)
    ref = torch.empty(B * N, H * 64, device="cuda", dtype=tdt)
    per = 16
    esz = ref.element_size()
    for b0 in range(0, B, per):
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr() + b0 * N * 3 * H * 64 * esz,
                                            ref.data_ptr() + b0 * N * H * 64 * esz, per, N, H, 64,
                                            0, 8, _stream()))
    out = torch.empty_like(ref)
    for _ in range(4):
        out.fill_(7.0)
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), B, N, H, 64, 0, 8,
                                            _stream()))
        torch.cuda.synchronize()
        assert torch.equal(out, ref), f"{(out != ref).sum().item()} elements differ"


def test_attention_spike(lib):
    """A key row that dominates one query forces the online-softmax rescale branch."""
    B, N, H = 1, 257, 1
    qkv = torch.randn(B * N, 3 * 64, device="cuda") * 0.5
    qkv[100, :64] = 2.0          # query 100
    qkv[200, 64:128] = 2.0       # key 200 in the 7th key tile -> max jumps late
    qkv = qkv.half()
    out = torch.empty(B * N, 64, device="cuda", dtype=torch.float16)
    _check(lib, lib.miclip_op_attention(0, qkv.data_ptr(), out.data_ptr(), B, N, H, 0, 0, 0,
                                        _stream()))
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, B, N, H, 0)
    assert (out.float() - ref).abs().max().item() < 6e-3


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("B,N,H,causal", [(2, 257, 16, 0), (1, 50, 3, 0), (3, 77, 2, 1),
                                          (1, 1, 1, 0), (2, 100, 2, 1), (1, 416, 2, 0),
                                          (5, 197, 4, 0)])
def test_attention_dh80(lib, dt, B, N, H, causal):
    """Head dim 80 (open_clip ViT-H/14: 16 heads on width 1280); scale 1/sqrt(80)."""
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N + H + causal + 80)
    qkv = (torch.randn(B * N, 3 * H * 80, device="cuda", generator=g) * 1.5).to(tdt)
    # canary past the output: the padding dims 80..95 must never be stored
    out = torch.full((B * N + 1, H * 80), 7.0, device="cuda", dtype=tdt)
    _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), B, N, H, 80, causal,
                                        0, _stream()))
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, B, N, H, causal, dh=80)
    err = (out[:B * N].float() - ref).abs().max().item()
    assert err < (4e-2 if dt == "bf16" else 6e-3), err
    assert bool((out[B * N] == 7.0).all())


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("B,N,H", [(2, 257, 16), (3, 160, 4), (1, 288, 2), (4, 200, 3), (64, 257, 16)])
def test_attention_dh80_two_phase_bitexact(lib, dt, B, N, H):
    """The two-phase head-dim-80 kernel (variant 2: Q by LDS-DMA, key tiles 0-3
    computed while the rest lands; the default outside N = 256..259) equals
    attention_kernel<80> (variant 1) bit for bit; outside its range (N < 129 or > 288,
    causal) variant 2 is refused, not replaced."""
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N + H + 801)
    qkv = (torch.randn(B * N, 3 * H * 80, device="cuda", generator=g) * 1.5).to(tdt)
    outs = []
    for v in (1, 2, 0):
        out = torch.full((B * N + 1, H * 80), 7.0, device="cuda", dtype=tdt)
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), B, N, H, 80, 0,
                                            v, _stream()))
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    if not 256 <= N <= 259:   # there the default is the pipelined kernel (variant 6)
        assert torch.equal(outs[1], outs[2])
    assert bool((outs[1][B * N] == 7.0).all())
    for bad_n, causal in ((100, 0), (300, 0), (257, 1)):
        x = torch.zeros(bad_n, 3 * 80, device="cuda", dtype=tdt)
        y = torch.zeros(bad_n, 80, device="cuda", dtype=tdt)
        assert lib.miclip_op_attention(code, x.data_ptr(), y.data_ptr(), 1, bad_n, 1, 80, causal, 2,
                                       _stream()) != 0


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("N", [256, 257, 258, 259])
def test_attention_dh80_pipelined(lib, dt, N):
    """The pipelined head-dim-80 kernel (variant 6, the default at N = 256..259: one
    workgroup walks hpw heads through a ring of three half-head K/V slots, the keys
    past the 8 full tiles on VALU, the ragged queries merged from 8 per-wave partials).
    Against the fp32 reference with hpw = 1 (16 heads) and hpw = 9 (2304 heads over 256
    CUs); every head's arithmetic is independent of hpw, so the whole batch must equal
    launches of 16 images (256 heads: hpw = 1) bit for bit, on every one of several
    repeats (a slot or partial race would vary run to run). Canary row past the output:
    the padding dims are never stored. Refused when causal or outside N = 256..259."""
    code, tdt = DT[dt]
    H = 16
    tol = 4e-2 if dt == "bf16" else 6e-3
    g = torch.Generator(device="cuda").manual_seed(N + 8080)
    small = (torch.randn(1 * N, 3 * H * 80, device="cuda", generator=g) * 1.5).to(tdt)
    out = torch.full((N + 1, H * 80), 7.0, device="cuda", dtype=tdt)
    _check(lib, lib.miclip_op_attention(code, small.data_ptr(), out.data_ptr(), 1, N, H, 80, 0, 6,
                                        _stream()))
    torch.cuda.synchronize()
    assert (out[:N].float() - _attn_ref(small, 1, N, H, 0, dh=80)).abs().max().item() < tol
    assert bool((out[N] == 7.0).all())
    B = 144                                  # 2304 heads: hpw = 9 on 256 CUs
    qkv = (torch.randn(B * N, 3 * H * 80, device="cuda", generator=g) * 1.5).to(tdt)
    ref = torch.empty(B * N, H * 80, device="cuda", dtype=tdt)
    per, esz = 16, ref.element_size()
    for b0 in range(0, B, per):
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr() + b0 * N * 3 * H * 80 * esz,
                                            ref.data_ptr() + b0 * N * H * 80 * esz, per, N, H, 80,
                                            0, 6, _stream()))
    torch.cuda.synchronize()
    want = _attn_ref(qkv[:4 * N], 4, N, H, 0, dh=80)
    assert (ref[:4 * N].float() - want).abs().max().item() < tol
    big = torch.empty(B * N + 1, H * 80, device="cuda", dtype=tdt)
    for _ in range(3):
        big.fill_(7.0)
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), big.data_ptr(), B, N, H, 80, 0, 0,
                                            _stream()))
        torch.cuda.synchronize()
        assert torch.equal(big[:B * N], ref), f"{(big[:B * N] != ref).sum().item()} elements differ"
        assert bool((big[B * N] == 7.0).all())
    # a short last workgroup: 143 images = 2288 heads, hpw = 9 over 255 workgroups, the
    # last one with nh = 2 (its ring and the partial merge stop early)
    Bs = 143
    short = torch.full((Bs * N + 1, H * 80), 7.0, device="cuda", dtype=tdt)
    _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), short.data_ptr(), Bs, N, H, 80, 0, 6,
                                        _stream()))
    torch.cuda.synchronize()
    assert torch.equal(short[:Bs * N], ref[:Bs * N]), \
        f"{(short[:Bs * N] != ref[:Bs * N]).sum().item()} elements differ"
    assert bool((short[Bs * N] == 7.0).all())
    for bad_n, causal in ((255, 0), (260, 0), (257, 1)):
        assert lib.miclip_op_attention(code, qkv.data_ptr(), big.data_ptr(), 1, bad_n, H, 80, causal,
                                       6, _stream()) != 0


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 16, 0), (1, 640, 2, 0), (3, 352, 3, 0),
                                          (2, 400, 2, 1), (1, 577, 3, 1)])
def test_attention_one_head_wave_counts(lib, dt, B, N, H, causal):
    """attention_kernel<64> (one head per workgroup, N > 320) on a forced number of waves
    (variants 10-16) equals the default (variant 1: one wave per chunk up to 16) bit
    for bit: a chunk's arithmetic does not depend on which wave runs it (causal too,
    where chunks carry unequal work). 17 is refused."""
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N + H + 1616 + causal)
    qkv = (torch.randn(B * N, 3 * H * 64, device="cuda", generator=g) * 1.5).to(tdt)
    outs = []
    for v in (1, 10, 12, 13, 16):
        out = torch.full((B * N + 1, H * 64), 7.0, device="cuda", dtype=tdt)
        _check(lib, lib.miclip_op_attention(code, qkv.data_ptr(), out.data_ptr(), B, N, H, 64,
                                            causal, v, _stream()))
        outs.append(out)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    assert bool((outs[0][B * N] == 7.0).all())
    ref = _attn_ref(qkv, B, N, H, causal)
    assert (outs[0][:B * N].float() - ref).abs().max().item() < (4e-2 if dt == "bf16" else 6e-3)
    assert lib.miclip_op_attention(code, qkv.data_ptr(), outs[0].data_ptr(), B, N, H, 64, causal,
                                   17, _stream()) != 0


@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("B,N,H,dh", [(3, 257, 16, 64), (2, 577, 16, 64), (5, 50, 12, 64),
                                      (2, 257, 16, 80), (1, 1, 1, 64), (2, 640, 2, 64), (1, 768, 2, 80),
                                      (7, 197, 3, 64), (1, 65, 5, 80)])
def test_attention_q0(lib, dt, B, N, H, dh):
    """CLS-query attention (the vision tower's last block): row 0 of each image
    against fp32 SDPA, compact [B, H*dh] output; rows past B untouched."""
    code, tdt = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N + H + dh)
    qkv = (torch.randn(B * N, 3 * H * dh, device="cuda", generator=g) * 1.5).to(tdt)
    out = torch.full((B + 1, H * dh), 7.0, device="cuda", dtype=tdt)
    _check(lib, lib.miclip_op_attention_q0(code, qkv.data_ptr(), out.data_ptr(), B, N, H, dh,
                                           _stream()))
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, B, N, H, 0, dh=dh).view(B, N, H * dh)[:, 0]
    err = (out[:B].float() - ref).abs().max().item()
    assert err < (4e-2 if dt == "bf16" else 6e-3), err
    assert bool((out[B] == 7.0).all())
    # out of range: N beyond the kernel's key capacity, head dims other than 64 / 80
    assert lib.miclip_op_attention_q0(code, qkv.data_ptr(), out.data_ptr(), 1, 769, H, dh,
                                      _stream()) != 0
    assert lib.miclip_op_attention_q0(code, qkv.data_ptr(), out.data_ptr(), 1, N, H, 96,
                                      _stream()) != 0


def test_attention_bad_head_dim(lib):
    x = torch.zeros(3 * 96, device="cuda", dtype=torch.float16)
    y = torch.zeros(96, device="cuda", dtype=torch.float16)
    assert lib.miclip_op_attention(0, x.data_ptr(), y.data_ptr(), 1, 1, 1, 96, 0, 0, _stream()) != 0


# The fp16 residual stream's rounding (clip/model.py:184-185 on half tensors):
# t = fp16(A.W^T + b), then the half add x + t. Integer-valued operands make the
# fp32 accumulation exact in any order, so every GEMM path -- the persistent
# kernel's transposed-accumulator epilogue (tile rows), its row tail, the other
# 256x256 schedules and the 128x128 kernel -- must match torch's own half-tensor
# arithmetic bit for bit (|A.W^T + b| reaches ~10^4, so fp16(.) really rounds).
@pytest.mark.parametrize("M,N,K,variant", [(16421, 1024, 1024, 0), (32896, 1024, 4096, 0),
                                           (16448, 1024, 1024, 259), (4096, 1024, 1024, 258),
                                           (1000, 768, 3072, 128), (300, 256, 192, 0)])
def test_gemm_residual_fp16_rounding_bitexact(lib, M, N, K, variant):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).half()
    W = torch.randint(-2, 3, (N, K), device="cuda", generator=g).half()
    bias = torch.randint(-8, 9, (N,), device="cuda", generator=g).float() * 0.25
    X0 = (torch.randn(M, N, device="cuda", generator=g) * 64).half()
    t = (A.double() @ W.double().t() + bias.double()).half()   # exact sum, one fp16 rounding
    ref = X0 + t                                      # torch half add
    X = X0.clone()
    _check(lib, lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), bias.data_ptr(), X.data_ptr(),
                                   M, N, K, 4, 0, variant, _stream()))
    torch.cuda.synchronize()
    assert torch.equal(X, ref), f"{(X != ref).sum().item()} elements differ"


# images [B, 3, R, R] -> patches [B*g*g, Kp] (conv1 as a GEMM operand, clip/model.py:217-219)
@pytest.mark.parametrize("B,R,P", [(3, 224, 32), (2, 224, 14), (2, 336, 14), (2, 224, 16),
                                   (2, 36, 9), (2, 42, 14), (1, 28, 28)])
@pytest.mark.parametrize("img_dt", [(3, torch.float32), (0, torch.float16), (1, torch.bfloat16)])
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
def test_im2col_band_vs_per_patch_and_unfold(lib, B, R, P, img_dt, dt):
    code, tdt = DT[dt]
    icode, idt = img_dt
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + R * 10 + P)
    img = torch.randn(B, 3, R, R, device="cuda", generator=g).to(idt)
    gg, K = R // P, 3 * P * P
    Kp = (K + 63) // 64 * 64
    # torch reference: each patch's (c, ky, kx) values in that order, zero pad to Kp
    ref = torch.zeros(B * gg * gg, Kp, device="cuda", dtype=tdt)
    ref[:, :K] = (img.float().reshape(B, 3, gg, P, gg, P).permute(0, 2, 4, 1, 3, 5)
                  .reshape(B * gg * gg, K).to(tdt))
    outs = []
    for variant in (0, 1):
        # NaN-filled (pad columns must be written) with a canary row past the end
        buf = torch.full((B * gg * gg + 1, Kp), float("nan"), device="cuda", dtype=tdt)
        _check(lib, lib.miclip_op_im2col(code, icode, img.data_ptr(), buf.data_ptr(), B, R, P, Kp,
                                         variant, _stream()))
        torch.cuda.synchronize()
        assert torch.isnan(buf[-1].float()).all(), "wrote past the end"
        outs.append(buf[:-1])
    assert torch.equal(outs[0].view(torch.int16), ref.view(torch.int16))
    assert torch.equal(outs[1].view(torch.int16), ref.view(torch.int16))
    # refusals: bad variant, Kp below 3*P*P, R not a multiple of P
    assert lib.miclip_op_im2col(code, icode, img.data_ptr(), outs[0].data_ptr(), B, R, P, Kp, 2,
                                _stream()) != 0
    assert lib.miclip_op_im2col(code, icode, img.data_ptr(), outs[0].data_ptr(), B, R, P, K - 1, 0,
                                _stream()) != 0
    assert lib.miclip_op_im2col(code, icode, img.data_ptr(), outs[0].data_ptr(), B, R + 1, P, Kp, 0,
                                _stream()) != 0
