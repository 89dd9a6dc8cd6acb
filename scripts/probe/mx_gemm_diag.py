"""Diagnostic: fp8 MX GEMM error structure against dequantised-operand references."""
import ctypes, sys, os
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "aihab-clip_amd"))
from miclip import _lib
from oracle import mx_oracle
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_mx import _blocky, _quant_gpu

lib = _lib.load_library()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for (M, N, K, blocky) in [(300, 256, 256, True), (300, 256, 256, False), (512, 768, 1280, True)]:
    if blocky:
        A = _blocky(M, K, M * 3 + K); W = _blocky(N, K, N * 5 + K) * 0.05
    else:
        g = np.random.default_rng(1)
        A = g.standard_normal((M, K)).astype(np.float32); W = (g.standard_normal((N, K)) * 0.05).astype(np.float32)
    qa, sa = _quant_gpu(lib, A); qw, sw = _quant_gpu(lib, W)
    C = torch.empty(M, N, dtype=torch.float32, device="cuda")
    bias = torch.zeros(N, device="cuda")
    C16 = torch.empty(M, N, dtype=torch.float16, device="cuda")
    assert lib.miclip_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                 C16.data_ptr(), None, M, N, K, 0, 0, s) == 0
    torch.cuda.synchronize()
    qA, EA = mx_oracle.quantize(A); qW, EW = mx_oracle.quantize(W)
    Ad = mx_oracle.dequantize(qA, EA).astype(np.float64); Wd = mx_oracle.dequantize(qW, EW).astype(np.float64)
    ref = Ad @ Wd.T
    got = C16.double().cpu().numpy()
    err = np.abs(got - ref); rel = err / (np.abs(Ad) @ np.abs(Wd).T + 1e-30)
    i, j = np.unravel_index(np.argmax(err - np.abs(ref) * 2 ** -10), err.shape)
    print(f"M{M} N{N} K{K} blocky={blocky}: max err {err.max():.3e}, max err/sum|ab| {rel.max():.3e}, "
          f"worst at ({i},{j}) got {got[i,j]:.6f} ref {ref[i,j]:.6f}")
    # per-k-block contribution check at the worst element: recompute with one block's scale doubled/halved
    contrib = (Ad[i] * Wd[j]).reshape(-1, 32).sum(1)
    print("   block contributions:", np.round(contrib, 4)[:16], " diff", got[i, j] - ref[i, j])
    # flush e4m3 subnormals
    def ftz(q, E):
        qq = q.copy(); sub = ((qq & 0x78) == 0) & ((qq & 7) != 0); qq[sub] = qq[sub] & 0x80
        return mx_oracle.dequantize(qq, E).astype(np.float64)
    ref2 = ftz(qA, EA) @ ftz(qW, EW).T
    print(f"   FTZ-subnormal ref: max err {np.abs(got - ref2).max():.3e}")
