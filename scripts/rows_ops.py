#!/usr/bin/env python
"""Row plans of the persistent GEMM, op level, interleaved: every variant of every
shape timed in R rounds (HIP events, random operands), median per (shape, variant).
Shapes: the ViT-L/14 block GEMMs at B images per GPU (M = 257 B) and the ViT-B/32
bs=256 ones (M = 12 800). Prints one JSON line per (shape, variant).
    rows_ops.py [--batches 256,128,64,32,16] [--variants 259,192,129,130,0] [--rounds 5]
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
    ap.add_argument("--batches", default="256,128,64,32,16")
    ap.add_argument("--variants", default="259,192,129,130,0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--c2", action="store_true", help="also the ViT-B/32 bs=256 shapes")
    args = ap.parse_args()
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = []
    for b in (int(x) for x in args.batches.split(",")):
        M, W = 257 * b, 1024
        shapes += [(f"L14b{b}_qkv", M, 3 * W, W, 0), (f"L14b{b}_out", M, W, W, 4),
                   (f"L14b{b}_fc", M, 4 * W, W, 0), (f"L14b{b}_proj", M, W, 4 * W, 4)]
    if args.c2:
        M, W = 12800, 768
        shapes += [("B32_qkv", M, 3 * W, W, 0), ("B32_out", M, W, W, 4), ("B32_fc", M, 4 * W, W, 0),
                   ("B32_proj", M, W, 4 * W, 4)]
    Mmax = max(sh[1] for sh in shapes)
    A = (torch.randn(Mmax, 4096, device="cuda", generator=g) * 0.5).half()
    Wt = (torch.randn(4096, 4096, device="cuda", generator=g) * 0.02).half()
    bias = torch.randn(4096, device="cuda", generator=g) * 0.02
    C = torch.empty(Mmax, 4096, device="cuda", dtype=torch.float16)
    variants = [int(v) for v in args.variants.split(",")]
    a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for _ in range(args.rounds):
        for name, M, N, K, epi in shapes:
            for v in variants:
                def fn():
                    rc = lib.miclip_op_gemm(0, A.data_ptr(), Wt.data_ptr(), bias.data_ptr(),
                                            C.data_ptr(), M, N, K, epi, 0, v, s)
                    assert rc == 0, lib.miclip_last_error()
                fn()
                a.record()
                for _ in range(args.iters):
                    fn()
                b_.record()
                torch.cuda.synchronize()
                res.setdefault((name, M, N, K, v), []).append(a.elapsed_time(b_) / args.iters)
    for (name, M, N, K, v), ts in res.items():
        ms = statistics.median(ts)
        print(json.dumps(dict(shape=name, M=M, N=N, K=K, variant=v, ms=round(ms, 4),
                              spread=round((max(ts) - min(ts)) / ms, 3),
                              tflops=round(2.0 * M * N * K / ms / 1e9, 1))), flush=True)


if __name__ == "__main__":
    main()
