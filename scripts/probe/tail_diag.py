import ctypes, sys, os, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "aihab-clip_amd"))
from miclip import _lib
lib = _lib.load_library()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
M, N, K = 16448, 1024, 1024
g = torch.Generator(device="cuda").manual_seed(1)
A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
bias = torch.randn(N, device="cuda", generator=g) * 0.1
def run(epi, act, v):
    C = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == 2 else torch.float16)
    assert lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(), M, N, K, epi, act, v, s) == 0
    torch.cuda.synchronize()
    return C
NT = 1 << 16
f32 = run(2, 0, 258)
for v in (258, 260):
    t1, t2, n1, n2 = run(0, 1, v), run(0, 1, v), run(0, 1, v | NT), run(0, 1, v | NT)
    print(v, "tail-tail", int((t1 != t2).sum()), "nt-nt", int((n1 != n2).sum()), "tail-nt", int((t1 != n1).sum()))
    idx = (t1 != n1).nonzero()
    for r, c in idx[:4].tolist():
        x = f32[r, c].item()
        print("  ", r, c, "pre", repr(x), x.hex() if hasattr(x, 'hex') else '', "tail", t1[r, c].item(), "nt", n1[r, c].item())
    # same rows inside the DP region: does the DP path agree with itself at other rows?
