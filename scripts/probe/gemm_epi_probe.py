#!/usr/bin/env python
"""Persistent GEMM (variant 0 = the launcher's default) at M = 65792, K = 1024 for
N in 2304 / 3072 / 4096: plain store (epi 0, act 0) against the folded-LN store
(miclip_op_gemm_ln, act 0), 3 interleaved rounds, fresh random operands.
Prints ms and us per round of 256 tiles."""
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


lib = _lib.load_library()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
g = torch.Generator(device="cuda").manual_seed(0)
M, K = 65792, 1024
A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
stats = torch.stack([torch.zeros(M, device="cuda"), torch.ones(M, device="cuda")], 1).contiguous()
for r in range(3):
    for N in (2304, 3072, 4096):
        W = (torch.randn(N, K, device="cuda", generator=g) * 0.02).half()
        bias = torch.randn(N, device="cuda", generator=g) * 0.02
        cs = torch.randn(N, device="cuda", generator=g) * 0.02
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        rounds = -(-((M // 256) * (N // 256)) // 256)
        for kind in ("store", "ln"):
            if kind == "store":
                def fn():
                    assert lib.miclip_op_gemm(0, A.data_ptr(), W.data_ptr(), bias.data_ptr(), C.data_ptr(),
                                              M, N, K, 0, 0, 0, s) == 0
            else:
                def fn():
                    assert lib.miclip_op_gemm_ln(0, A.data_ptr(), W.data_ptr(), bias.data_ptr(), cs.data_ptr(),
                                                 stats.data_ptr(), C.data_ptr(), M, N, K, 0, 0, s) == 0
            ms = timeit(fn)
            print(json.dumps(dict(round=r, N=N, epi=kind, ms=round(ms, 4), rounds=rounds,
                                  us_per_round=round(ms * 1000 / rounds, 2),
                                  tflops=round(2.0 * M * N * K / ms / 1e9, 1))), flush=True)
        del W, C
