#!/usr/bin/env python
"""MX-fp8 GEMM at the ViT-H-14 bs=512 split shapes (M = 65792): time per epilogue
(fp16 store, MX-fp8 out with GELU / without, fp16 residual) to size the c_fc
epilogue against the main loop. Random operands, HIP events on torch's stream."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))
import torch  # noqa: E402
from miclip import _lib  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    M, W = int(os.environ.get("M", "65792")), 1280
    shapes = [("qkv", 3 * W, W), ("fc", 4 * W, W), ("proj", W, 4 * W)]
    rounds = int(os.environ.get("ROUNDS", "2"))
    for _ in range(rounds):
        for name, N, K in shapes:
            a32 = torch.randn(M, K, device="cuda", generator=g)
            w32 = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
            qa = torch.empty(M, K, device="cuda", dtype=torch.uint8)
            sa = torch.empty(lib.miclip_mx_scale_bytes(M, K), device="cuda", dtype=torch.uint8)
            qw = torch.empty(N, K, device="cuda", dtype=torch.uint8)
            sw = torch.empty(lib.miclip_mx_scale_bytes(N, K), device="cuda", dtype=torch.uint8)
            assert lib.miclip_op_quant_mx(a32.data_ptr(), 0, M, K, qa.data_ptr(), sa.data_ptr(), s) == 0
            assert lib.miclip_op_quant_mx(w32.data_ptr(), 0, N, K, qw.data_ptr(), sw.data_ptr(), s) == 0
            del a32, w32
            bias = torch.randn(N, device="cuda", generator=g) * 0.1
            c16 = torch.empty(M, N, device="cuda", dtype=torch.float16)
            cq = torch.empty(M, N, device="cuda", dtype=torch.uint8)
            cs = torch.empty(lib.miclip_mx_scale_bytes(M, N), device="cuda", dtype=torch.uint8)
            cases = [("store", 0, 0, c16, None), ("store_gelu", 0, 2, c16, None),
                     ("mx", 5, 0, cq, cs), ("mx_gelu", 5, 2, cq, cs), ("mx_gelu_tanh", 5, 3, cq, cs), ("resid", 1, 0, c16, None)]
            for tag, epi, act, C, CS in cases:
                if name != "fc" and tag in ("store_gelu", "mx_gelu", "mx_gelu_tanh"):
                    continue

                def fn():
                    rc = lib.miclip_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(),
                                               bias.data_ptr(), C.data_ptr(), CS.data_ptr() if CS is not None else None,
                                               M, N, K, epi, act, s)
                    assert rc == 0, lib.miclip_last_error()
                ms = timeit(fn)
                print(json.dumps(dict(op=f"mx_{name}", epi=tag, M=M, N=N, K=K, ms=round(ms, 4),
                                      tflops=round(2.0 * M * N * K / ms / 1e9, 1))), flush=True)
            del qa, sa, qw, sw, c16, cq, cs


if __name__ == "__main__":
    main()
