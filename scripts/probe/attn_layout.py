#!/usr/bin/env python
"""Layout probe for the x8 attention at N = 257: the QKV buffer token-major (the
projection's [B N, 3 D], variant 8) against head-major ([B][H][3][N][64], each
head's Q, K and V rows contiguous, variant 24). Same arithmetic: outputs must be
bitwise equal; then interleaved timing rounds (HBM access pattern only differs).

Usage: python scripts/probe/attn_layout.py [B] [N]
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 257
    H, dh = 16, 64
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    tm = torch.randn(B * N, 3 * H * dh, device="cuda", generator=g).half()
    hm = tm.view(B, N, 3, H, dh).permute(0, 3, 2, 1, 4).contiguous()
    o8 = torch.full((B * N, H * dh), float("nan"), device="cuda", dtype=torch.float16)
    o24 = o8.clone()
    assert lib.miclip_op_attention(0, tm.data_ptr(), o8.data_ptr(), B, N, H, dh, 0, 8, s) == 0
    assert lib.miclip_op_attention(0, hm.data_ptr(), o24.data_ptr(), B, N, H, dh, 0, 24, s) == 0
    torch.cuda.synchronize()
    eq = torch.equal(o8, o24)
    print(json.dumps({"check": "head-major vs token-major bitwise", "equal": eq}), flush=True)
    assert eq
    fl = 4.0 * B * H * N * N * dh
    res = {8: [], 24: []}
    for rnd in range(5):
        for v, buf in ((8, tm), (24, hm)):
            def fa():
                assert lib.miclip_op_attention(0, buf.data_ptr(), o8.data_ptr(), B, N, H, dh, 0, v, s) == 0
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
    for v in res:
        ms = sorted(res[v])
        print(json.dumps({"op": "attention", "layout": "token-major" if v == 8 else "head-major",
                          "B": B, "N": N, "variant": v, "ms": [round(x, 4) for x in res[v]],
                          "median_ms": round(ms[len(ms) // 2], 4),
                          "tflops_best": round(fl / ms[0] / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
