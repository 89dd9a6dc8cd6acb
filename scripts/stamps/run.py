#!/usr/bin/env python
"""In-kernel cycle stamps of the persistent GEMM and the x8 attention kernel.

Loads a diagnostic library built by `make stamps` (the library's objects with
gemm.hip or attention.hip recompiled under MICLIP_STAMPS, common.h), runs one
launch at the ViT-L/14 bs=256 shapes on random operands and prints, per
segment, the mean s_memtime cycles per wave, the share of the wave's lifetime
and the effective shader clock (s_memtime cycles / s_memrealtime ticks at
100 MHz). The stamps cost cycles of their own (guide: ~+11 % with one per
segment), so shares, not absolute times, are the result.

  python scripts/stamps/run.py gemm [--shape fc|qkv|out|proj] [--m 32896]
  python scripts/stamps/run.py attn [--b 128] [--n 257]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SEGS = {
    "gemm": ["tile_top", "main_loop", "boundary", "epilogue", "row_tail", "epi_math_stage",
             "epi_barrier", "epi_readback_store"],
    "gemm_phases": ["outside_k_loop", "frag_reads", "dma_issue", "lgkm_wait", "barrier_pre_mfma",
                    "mfma_issue", "vmcnt_wait", "barrier_close"],
    "attn": ["kv_load_wait", "chunk", "store", "ragged", "close_barrier", "merge", "dma_issue",
             "q_load_and_wait"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel", choices=["gemm", "attn"])
    ap.add_argument("--shape", default="fc")
    ap.add_argument("--m", type=int, default=32896)
    ap.add_argument("--b", type=int, default=128)
    ap.add_argument("--n", type=int, default=257)
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--null", action="store_true", help="gemm: the no-output epilogue (epi 3)")
    ap.add_argument("--phases", action="store_true",
                    help="gemm: segment names of the K-loop phase build (libstamp_gemm_kphase.so)")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.environ.get("STAMP_LIB") or
                      os.path.join(ROOT, "build", "stamps", f"libstamp_{args.kernel}.so"))
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    W = 1024
    if args.kernel == "gemm":
        N, K = {"qkv": (3 * W, W), "fc": (4 * W, W), "out": (W, W), "proj": (W, 4 * W)}[args.shape]
        M = args.m
        A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
        Wt = (torch.randn(N, K, device="cuda", generator=g) * 0.02).half()
        bias = torch.randn(N, device="cuda", generator=g) * 0.02
        colsum = torch.randn(N, device="cuda", generator=g) * 0.02
        st = torch.stack([torch.randn(M, device="cuda", generator=g),
                          torch.rand(M, device="cuda", generator=g) + 0.5], 1).contiguous()
        C = torch.empty(M, N, device="cuda", dtype=torch.float16)
        flops = 2.0 * M * N * K
        if args.null:
            Cf = torch.empty(M, N, device="cuda", dtype=torch.float32)
            fn = lambda: lib.miclip_op_gemm(0, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Wt.data_ptr()),
                                            ctypes.c_void_p(bias.data_ptr()), ctypes.c_void_p(Cf.data_ptr()),
                                            M, N, K, 3, 0, 0, s)
        elif args.shape in ("qkv", "fc"):
            act = int(args.shape == "fc")
            fn = lambda: lib.miclip_op_gemm_ln(0, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Wt.data_ptr()),
                                               ctypes.c_void_p(bias.data_ptr()), ctypes.c_void_p(colsum.data_ptr()),
                                               ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(C.data_ptr()),
                                               M, N, K, act, 0, s)
        else:
            fn = lambda: lib.miclip_op_gemm(0, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Wt.data_ptr()),
                                            ctypes.c_void_p(bias.data_ptr()), ctypes.c_void_p(C.data_ptr()),
                                            M, N, K, 4, 0, 0, s)
        wpb = 8
    else:
        B, Nq, H = args.b, args.n, 16
        qkv = (torch.randn(B * Nq, 3 * H * 64, device="cuda", generator=g)).half()
        out = torch.empty(B * Nq, H * 64, device="cuda", dtype=torch.float16)
        flops = 4.0 * B * H * Nq * Nq * 64
        fn = lambda: lib.miclip_op_attention(0, ctypes.c_void_p(qkv.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                             B, Nq, H, 64, 0, 8, s)
        wpb = 8
    for _ in range(args.warm):
        assert fn() == 0
    torch.cuda.synchronize()
    assert lib.miclip_stamps_clear(s) == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    assert fn() == 0
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1])
    words = lib.miclip_stamps_words()
    buf = np.zeros(words, dtype=np.uint64)
    assert lib.miclip_stamps_read(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))) == 0
    rec = buf[: words // 10 * 10].reshape(-1, 10)
    rec = rec[rec[:, 8] > 0].astype(np.float64)       # waves that ran
    tot = rec[:, 8]
    clock = tot / (rec[:, 9] / 100e6)                   # cycles per second
    names = SEGS["gemm_phases" if args.kernel == "gemm" and args.phases else args.kernel]
    segs = {n: dict(mean_cycles=round(float(rec[:, i].mean())),
                    share=round(float(rec[:, i].sum() / tot.sum()), 4))
            for i, n in enumerate(names)}
    print(json.dumps(dict(kernel=args.kernel, shape=args.shape if args.kernel == "gemm" else f"B{args.b}xN{args.n}",
                          waves=int(len(rec)), ms=round(ms, 4), tflops=round(flops / ms / 1e9, 1),
                          wave_cycles_mean=round(float(tot.mean())), wave_cycles_max=round(float(tot.max())),
                          clock_ghz_mean=round(float(clock.mean()) / 1e9, 3),
                          clock_ghz_min=round(float(clock.min()) / 1e9, 3),
                          segments=segs), indent=1))


if __name__ == "__main__":
    main()
