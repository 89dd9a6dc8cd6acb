#!/usr/bin/env python
"""Time the pieces of the CLS-only last vision block (capi.hip run_block cls_only)
at ViT-L/14 shapes for `--items` images: CLS-query attention, and the M = items
out-proj / c_fc / c_proj GEMMs through the op entry points (variants as given)."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from bench_ops import timeit  # noqa: E402
from miclip import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=128)
    ap.add_argument("--tokens", type=int, default=257)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    B, N, W = args.items, args.tokens, args.width
    H = W // 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * N, 3 * W, device="cuda", generator=g).half()
    o = torch.empty(B, W, device="cuda", dtype=torch.float16)
    ms = timeit(lambda: lib.miclip_op_attention_q0(0, qkv.data_ptr(), o.data_ptr(), B, N, H, 64, s),
                args.iters)
    print(json.dumps(dict(op="attention_q0", B=B, N=N, ms=round(ms, 4),
                          gbs=round(B * N * 2 * W * 2 / ms / 1e6, 1))), flush=True)
    A = (torch.randn(B, 4 * W, device="cuda", generator=g) * 0.5).half()
    Wt = (torch.randn(4 * W, 4 * W, device="cuda", generator=g) * 0.02).half()
    bias = torch.randn(4 * W, device="cuda", generator=g) * 0.02
    X16 = torch.randn(B, W, device="cuda", generator=g).half()
    C16 = torch.empty(B, 4 * W, device="cuda", dtype=torch.float16)
    for v in [int(x) for x in args.variants.split(",")]:
        for name, Nn, K, epi, act in (("out", W, W, 4, 0), ("fc", 4 * W, W, 0, 1), ("proj", W, 4 * W, 4, 0)):
            a = A[:, :K].contiguous()
            w = Wt[:Nn, :K].contiguous()
            C = X16 if epi == 4 else C16
            fn = lambda: lib.miclip_op_gemm(0, a.data_ptr(), w.data_ptr(), bias.data_ptr(), C.data_ptr(),
                                            B, Nn, K, epi, act, v, s)
            assert fn() == 0, lib.miclip_last_error()
            ms = timeit(fn, args.iters)
            print(json.dumps(dict(op=f"gemm_{name}", variant=v, M=B, N=Nn, K=K, ms=round(ms, 4),
                                  tflops=round(2.0 * B * Nn * K / ms / 1e9, 1),
                                  gbs=round(2.0 * Nn * K / ms / 1e6, 1))), flush=True)


if __name__ == "__main__":
    main()
