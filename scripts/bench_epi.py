#!/usr/bin/env python
"""Price each GEMM epilogue at the ViT-L/14 bs=256 shapes (one process, HIP events).

For M = 65792 and (N, K) of QKV / c_fc / out-proj / c_proj it times the same
persistent 256x256 kernel with: no output (epi 3, the main loop alone), the plain
store, the store + QuickGELU, the folded-LN store (+QuickGELU) and the fp16
residual epilogue, interleaved `--rounds` times on random operands.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))

import torch  # noqa: E402

from miclip import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="qkv,fc,out,proj")
    ap.add_argument("--m", type=int, default=256 * 257, help="rows (32896 = one splits=2 half)")
    args = ap.parse_args()
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    M, W = args.m, 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    A = (torch.randn(M, 4 * W, device="cuda", generator=g) * 0.5).half()
    Wt = (torch.randn(4 * W, 4 * W, device="cuda", generator=g) * 0.02).half()
    bias = torch.randn(4 * W, device="cuda", generator=g) * 0.02
    C = torch.empty(M, 4 * W, device="cuda", dtype=torch.float16)
    X16 = torch.randn(M, W, device="cuda", generator=g).half()
    st = torch.stack([torch.randn(M, device="cuda", generator=g),
                      torch.rand(M, device="cuda", generator=g) + 0.5], 1).contiguous()
    Cf = torch.empty(M, 4 * W, device="cuda", dtype=torch.float32)
    shapes = {"qkv": (3 * W, W), "fc": (4 * W, W), "out": (W, W), "proj": (W, 4 * W)}
    cases = []
    for name in args.shapes.split(","):
        N, K = shapes[name]
        a = A[:, :K].contiguous() if K != 4 * W else A
        w = Wt[:N, :K].contiguous()

        def mk(kind, N=N, K=K, a=a, w=w):
            if kind == "null":
                return lambda: lib.miclip_op_gemm(0, a.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                                  Cf.data_ptr(), M, N, K, 3, 0, 0, s)
            if kind in ("store", "gelu"):
                return lambda: lib.miclip_op_gemm(0, a.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                                  C.data_ptr(), M, N, K, 0, int(kind == "gelu"), 0, s)
            if kind in ("ln", "lngelu"):
                return lambda: lib.miclip_op_gemm_ln(0, a.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                                     bias.data_ptr(), st.data_ptr(), C.data_ptr(),
                                                     M, N, K, int(kind == "lngelu"), 0, s)
            return lambda: lib.miclip_op_gemm(0, a.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                              X16.data_ptr(), M, N, K, 4, 0, 0, s)
        kinds = {"qkv": ["null", "store", "ln"], "fc": ["null", "store", "gelu", "ln", "lngelu"],
                 "out": ["null", "resid"], "proj": ["null", "resid"]}[name]
        for k in kinds:
            cases.append((name, k, N, K, mk(k)))
    res = {}
    a_ev, b_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.rounds):
        for name, kind, N, K, fn in cases:
            for _ in range(3):
                assert fn() == 0, lib.miclip_last_error()
            torch.cuda.synchronize()
            a_ev.record()
            for _ in range(args.iters):
                fn()
            b_ev.record()
            torch.cuda.synchronize()
            res.setdefault((name, kind, N, K), []).append(a_ev.elapsed_time(b_ev) / args.iters)
    for (name, kind, N, K), ts in res.items():
        ms = statistics.median(ts)
        print(json.dumps(dict(shape=name, epilogue=kind, M=M, N=N, K=K, ms=round(ms, 4),
                              tflops=round(2.0 * M * N * K / ms / 1e9, 1),
                              runs=[round(t, 4) for t in ts])), flush=True)


if __name__ == "__main__":
    main()
