#!/usr/bin/env python
"""MX-fp8 GEMM launches at the ViT-H/14 shapes (C5) with M = 256 x 256 rows (whole
rounds of 256x256 tiles on 256 CUs) against M = 257 x 256 (one batch-split's rows
at B = 256: one more row-block, i.e. one more, nearly empty, round of tiles):
prints ms per launch for each M, interleaved over rounds.

Usage: python scripts/probe/mx_rounds.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))

import torch  # noqa: E402

from miclip import _lib  # noqa: E402


def main():
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    Ms = (65536, 65792)
    shapes = [("qkv", 3840, 1280, 0, 0), ("out", 1280, 1280, 1, 0), ("fc", 5120, 1280, 5, 2),
              ("proj", 1280, 5120, 1, 0)]

    def quant(rows, K):
        x = (torch.randn(rows, K, device="cuda", generator=g) * 0.5).half()
        q = torch.empty(rows, K, device="cuda", dtype=torch.uint8)
        sc = torch.empty(lib.miclip_mx_scale_bytes(rows, K), device="cuda", dtype=torch.uint8)
        assert lib.miclip_op_quant_mx(x.data_ptr(), 1, rows, K, q.data_ptr(), sc.data_ptr(), s) == 0
        return q, sc

    res = {}
    for name, N, K, epi, act in shapes:
        A, SA = quant(Ms[-1], K)
        W, SW = quant(N, K)
        bias = torch.randn(N, device="cuda", generator=g) * 0.1
        C = torch.randn(Ms[-1], N, device="cuda", generator=g).half()
        Cq = torch.empty(Ms[-1], N, device="cuda", dtype=torch.uint8)
        CS = torch.empty(max(lib.miclip_mx_scale_bytes(Ms[-1], N), 1), device="cuda", dtype=torch.uint8)
        for rnd in range(3):
            for M in Ms:
                SAm = SA   # the tiled scale plane of the first M rows is a prefix (256-row tiles)
                out = Cq if epi == 5 else C

                def f():
                    rc = lib.miclip_op_gemm_mx(A.data_ptr(), SAm.data_ptr(), W.data_ptr(), SW.data_ptr(),
                                               bias.data_ptr(), out.data_ptr(),
                                               CS.data_ptr() if epi == 5 else None, M, N, K, epi, act, s)
                    assert rc == 0, lib.miclip_last_error()
                for _ in range(3):
                    f()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                a.record()
                for _ in range(20):
                    f()
                b.record()
                torch.cuda.synchronize()
                res.setdefault((name, M), []).append(a.elapsed_time(b) / 20)
        for M in Ms:
            ms = res[(name, M)]
            print(json.dumps({"op": name, "M": M, "N": N, "K": K, "ms": [round(x, 4) for x in ms],
                              "tflops_best": round(2.0 * M * N * K / min(ms) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
