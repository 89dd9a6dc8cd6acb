"""Probe: run each op of the MX-fp8 ViT-H-14 layer 6 times on the same inputs
(one split's shapes: M = 128 x 257) and report any bitwise run-to-run change."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "aihab-clip_amd"), ROOT]
import torch
from miclip import _lib

lib = _lib.load_library()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
B, Ntok, W, H = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 257, 1280, 16
M = B * Ntok
g = torch.Generator(device="cuda").manual_seed(0)


def chk(rc):
    assert rc == 0, lib.miclip_last_error().decode()


def quant(x):
    R, K = x.shape
    q = torch.empty(R, K, dtype=torch.uint8, device="cuda")
    sc = torch.zeros(int(lib.miclip_mx_scale_bytes(R, K)), dtype=torch.uint8, device="cuda")
    chk(lib.miclip_op_quant_mx(x.data_ptr(), 1, R, K, q.data_ptr(), sc.data_ptr(), s))
    return q, sc


def rep(name, fn, outs, n=int(os.environ.get("REPS", "6"))):
    res = []
    for _ in range(n):
        for o in outs:
            o.zero_()
        fn()
        torch.cuda.synchronize()
        res.append([o.clone() for o in outs])
    bad = [i for i in range(1, n) if any(not torch.equal(a, b) for a, b in zip(res[i], res[0]))]
    detail = ""
    if bad:
        a, b = res[bad[0]][0], res[0][0]
        d = (a != b)
        detail = f" first differing run {bad[0]}: {d.sum().item()} elements, rows {torch.nonzero(d.view(d.shape[0], -1).any(1)).flatten()[:8].tolist()}"
    print(f"{name}: {'NONDETERMINISTIC' if bad else 'deterministic'} ({len(bad)} of {n - 1} runs differ){detail}", flush=True)


x16 = (torch.randn(M, W, device="cuda", generator=g) * 2).half()
gamma = torch.rand(W, device="cuda", generator=g) + 0.5
beta = torch.randn(W, device="cuda", generator=g) * 0.1
qa = torch.empty(M, W, dtype=torch.uint8, device="cuda")
sa = torch.zeros(int(lib.miclip_mx_scale_bytes(M, W)), dtype=torch.uint8, device="cuda")
rep("layernorm_mx", lambda: chk(lib.miclip_op_layernorm_mx(x16.data_ptr(), 1, gamma.data_ptr(), beta.data_ptr(),
                                                           qa.data_ptr(), sa.data_ptr(), M, W, s)), [qa, sa])
Wq = (torch.randn(3 * W, W, device="cuda", generator=g) * 0.03).half()
qw, sw = quant(Wq)
bias = torch.randn(3 * W, device="cuda", generator=g) * 0.1
qkv = torch.empty(M, 3 * W, device="cuda", dtype=torch.float16)
rep("gemm_mx qkv (epi 0)", lambda: chk(lib.miclip_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(),
                                                             bias.data_ptr(), qkv.data_ptr(), None, M, 3 * W, W, 0, 0, s)), [qkv])
o = torch.empty(M, W, device="cuda", dtype=torch.float16)
rep("attention dh80", lambda: chk(lib.miclip_op_attention(0, qkv.data_ptr(), o.data_ptr(), B, Ntok, H, 80, 0, 0, s)), [o])
Wo = (torch.randn(W, W, device="cuda", generator=g) * 0.03).half()
bo = torch.randn(W, device="cuda", generator=g) * 0.1
X = torch.empty_like(x16)
def outproj():
    X.copy_(x16)
    chk(lib.miclip_op_gemm(0, o.data_ptr(), Wo.data_ptr(), bo.data_ptr(), X.data_ptr(), M, W, W, 4, 0, 0, s))
rep("gemm out-proj fp16 residual", outproj, [X])
Wf = (torch.randn(4 * W, W, device="cuda", generator=g) * 0.03).half()
qf, sf = quant(Wf)
bf = torch.randn(4 * W, device="cuda", generator=g) * 0.1
Q = torch.empty(M, 4 * W, dtype=torch.uint8, device="cuda")
S = torch.zeros(int(lib.miclip_mx_scale_bytes(M, 4 * W)), dtype=torch.uint8, device="cuda")
rep("gemm_mx c_fc -> GELU -> MX (epi 5)", lambda: chk(lib.miclip_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qf.data_ptr(), sf.data_ptr(),
                                                                           bf.data_ptr(), Q.data_ptr(), S.data_ptr(), M, 4 * W, W, 5, 2, s)), [Q, S])
Wp = (torch.randn(W, 4 * W, device="cuda", generator=g) * 0.015).half()
qp, sp = quant(Wp)
bp = torch.randn(W, device="cuda", generator=g) * 0.1
X2 = torch.empty_like(x16)
def cproj():
    X2.copy_(x16)
    chk(lib.miclip_op_gemm_mx(Q.data_ptr(), S.data_ptr(), qp.data_ptr(), sp.data_ptr(), bp.data_ptr(), X2.data_ptr(), None,
                              M, W, 4 * W, 1, 0, s))
rep("gemm_mx c_proj residual (epi 1)", cproj, [X2])
