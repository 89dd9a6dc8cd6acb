"""Probe: each op of the MX-fp8 layer run on two streams at once (independent
operands, like the encode's two batch parts), repeated; any bitwise change
against a solo run of the same op means a race that co-residency exposes.
Usage: det_concurrent.py [B] (M = B x 257 rows per stream, ViT-H-14 widths)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "aihab-clip_amd"), ROOT]
import torch
from miclip import _lib

lib = _lib.load_library()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
W = int(os.environ.get("WIDTH", "1280"))
M = B * 257
REPS = int(os.environ.get("REPS", "8"))
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
g = torch.Generator(device="cuda").manual_seed(0)


def chk(rc):
    assert rc == 0, lib.miclip_last_error().decode()


def quant(x, st):
    R, K = x.shape
    q = torch.empty(R, K, dtype=torch.uint8, device="cuda")
    sc = torch.zeros(int(lib.miclip_mx_scale_bytes(R, K)), dtype=torch.uint8, device="cuda")
    chk(lib.miclip_op_quant_mx(x.data_ptr(), 1, R, K, q.data_ptr(), sc.data_ptr(), ctypes.c_void_p(st.cuda_stream)))
    return q, sc


def run(name, make):
    """make(k) -> (fn(stream_handle), outs) for operand set k."""
    sets = [make(k) for k in range(2)]
    torch.cuda.synchronize()
    ref = []
    for fn, outs in sets:   # solo runs
        for o in outs:
            o.zero_()
        fn(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        ref.append([o.clone() for o in outs])
    bad = 0
    for _ in range(REPS):
        for fn, outs in sets:
            for o in outs:
                o.zero_()
        torch.cuda.synchronize()
        for k, (fn, outs) in enumerate(sets):
            fn(ctypes.c_void_p(streams[k].cuda_stream))
        torch.cuda.synchronize()
        for k, (fn, outs) in enumerate(sets):
            if any(not torch.equal(a, b) for a, b in zip(outs, ref[k])):
                bad += 1
                d = outs[0] != ref[k][0]
                rows = torch.nonzero(d.view(d.shape[0], -1).any(1)).flatten()
                print(f"  {name} set {k}: {d.sum().item()} elements differ, rows {rows[:6].tolist()} ... {rows.numel()} rows", flush=True)
    print(f"{name}: {'RACE' if bad else 'ok'} ({bad} of {2 * REPS} concurrent results differ)", flush=True)


def mk_ln(k):
    x16 = (torch.randn(M, W, device="cuda", generator=g) * 2).half()
    gamma = torch.rand(W, device="cuda", generator=g) + 0.5
    beta = torch.randn(W, device="cuda", generator=g) * 0.1
    qa = torch.empty(M, W, dtype=torch.uint8, device="cuda")
    sa = torch.zeros(int(lib.miclip_mx_scale_bytes(M, W)), dtype=torch.uint8, device="cuda")
    return (lambda s: chk(lib.miclip_op_layernorm_mx(x16.data_ptr(), 1, gamma.data_ptr(), beta.data_ptr(),
                                                     qa.data_ptr(), sa.data_ptr(), M, W, s)), [qa, sa])


def mk_gemm(N, K, epi, act):
    def mk(k):
        a = (torch.randn(M, K, device="cuda", generator=g)).half()
        w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
        qa, sa = quant(a, torch.cuda.current_stream())
        qw, sw = quant(w, torch.cuda.current_stream())
        bias = torch.randn(N, device="cuda", generator=g) * 0.1
        if epi == 5:
            C = torch.empty(M, N, dtype=torch.uint8, device="cuda")
            CS = torch.zeros(int(lib.miclip_mx_scale_bytes(M, N)), dtype=torch.uint8, device="cuda")
            outs = [C, CS]
        else:
            C = torch.empty(M, N, dtype=torch.float16, device="cuda")
            CS = None
            outs = [C]
        X0 = torch.randn(M, N, device="cuda", generator=g).half()

        def fn(s):
            if epi == 1:
                C.copy_(X0)
                torch.cuda.current_stream().synchronize()
            chk(lib.miclip_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                      C.data_ptr(), CS.data_ptr() if CS is not None else None, M, N, K, epi, act, s))
        return fn, outs
    return mk


def mk_f16(N, K):
    def mk(k):
        a = (torch.randn(M, K, device="cuda", generator=g)).half()
        w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
        bias = torch.randn(N, device="cuda", generator=g) * 0.1
        X0 = torch.randn(M, N, device="cuda", generator=g).half()
        X = torch.empty_like(X0)

        def fn(s):
            X.copy_(X0)
            torch.cuda.current_stream().synchronize()
            chk(lib.miclip_op_gemm(0, a.data_ptr(), w.data_ptr(), bias.data_ptr(), X.data_ptr(), M, N, K, 4, 0, 0, s))
        return fn, [X]
    return mk


CASES = os.environ.get("CASES", "ln,qkv,fc,proj,f16").split(",")
if "ln" in CASES: run("layernorm_mx", mk_ln)
if "qkv" in CASES: run("gemm_mx qkv epi0", mk_gemm(3 * W, W, 0, 0))
if "fc" in CASES: run("gemm_mx fc epi5 gelu", mk_gemm(4 * W, W, 5, 3))
if "proj" in CASES: run("gemm_mx proj epi1", mk_gemm(W, 4 * W, 1, 0))
if "proj0" in CASES: run("gemm_mx N=W K=4W epi0", mk_gemm(W, 4 * W, 0, 0))
if "fc1" in CASES: run("gemm_mx N=4W K=W epi1", mk_gemm(4 * W, W, 1, 0))
if "f16" in CASES: run("gemm f16 out-proj residual", mk_f16(W, W))
