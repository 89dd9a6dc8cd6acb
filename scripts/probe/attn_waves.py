#!/usr/bin/env python
"""One-head-per-workgroup attention (attention_kernel<64>) at N = 577 (ViT-L/14@336, C4)
with the wave count forced (variant 10..16 = that many waves; variant 1 = the default
count): outputs compared bitwise with variant 1, then interleaved timing rounds.

Usage: python scripts/probe/attn_waves.py [B] [N] [variants, comma list]
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 577
    vs = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,10,12,14,16").split(",")]
    H, dh = 16, 64
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    for dt, code in ((torch.float16, 0), (torch.bfloat16, 1)):
        qkv = torch.randn(B * N, 3 * H * dh, device="cuda", generator=g).to(dt)
        outs = {}
        for v in vs:
            o = torch.full((B * N, H * dh), float("nan"), device="cuda", dtype=dt)
            rc = lib.miclip_op_attention(code, qkv.data_ptr(), o.data_ptr(), B, N, H, dh, 0, v, s)
            assert rc == 0, (v, lib.miclip_last_error())
            outs[v] = o
        torch.cuda.synchronize()
        for v in vs:
            eq = torch.equal(outs[v], outs[vs[0]])
            print(json.dumps({"check": "bitwise vs variant %d" % vs[0], "dtype": str(dt), "variant": v,
                              "equal": eq}), flush=True)
            assert eq, v
    qkv = torch.randn(B * N, 3 * H * dh, device="cuda", generator=g).half()
    o = torch.empty(B * N, H * dh, device="cuda", dtype=torch.float16)
    fl = 4.0 * B * H * N * N * dh
    res = {v: [] for v in vs}
    for rnd in range(4):
        for v in vs:
            def fa():
                assert lib.miclip_op_attention(0, qkv.data_ptr(), o.data_ptr(), B, N, H, dh, 0, v, s) == 0
            for _ in range(3):
                fa()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for _ in range(20):
                fa()
            b.record()
            torch.cuda.synchronize()
            res[v].append(a.elapsed_time(b) / 20)
    for v in vs:
        ms = sorted(res[v])
        print(json.dumps({"op": "attention", "B": B, "N": N, "variant": v,
                          "ms": [round(x, 4) for x in res[v]], "median_ms": round(ms[len(ms) // 2], 4),
                          "tflops_best": round(fl / ms[0] / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
