#!/usr/bin/env python
"""Same-process A/B of two builds of libmiclip.so on the head-dim-80 attention and the
MX LayerNorm at the C5 (ViT-H/14 bs=512, two streams) shapes: outputs compared
bitwise, then interleaved timing rounds. Used for layout-only changes (LDS swizzles),
which must not change a single output bit.

Usage: python scripts/probe/prev_vs_new.py PREV_LIB [NEW_LIB]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))

import torch  # noqa: E402

from miclip import _lib  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
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
    prev = _lib.load_library(sys.argv[1])
    new = _lib.load_library(sys.argv[2] if len(sys.argv) > 2 else _lib.LIB_PATH)
    libs = {"prev": prev, "new": new}
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    B, N, H, dh = 256, 257, 16, 80
    W = H * dh
    qkv = torch.randn(B * N, 3 * W, device="cuda", generator=g).half()
    outs = {}
    for name, lib in libs.items():
        for v in (0, 1):
            o = torch.full((B * N, W), float("nan"), device="cuda", dtype=torch.float16)
            assert lib.miclip_op_attention(0, qkv.data_ptr(), o.data_ptr(), B, N, H, dh, 0, v, s) == 0
            outs[(name, v)] = o
    torch.cuda.synchronize()
    for v in (0, 1):
        print(json.dumps({"check": "attention dh80 prev == new", "variant": v,
                          "equal": torch.equal(outs[("prev", v)], outs[("new", v)])}), flush=True)
    R, D = B * N, W
    x = (torch.randn(R, D, device="cuda", generator=g) * 3 + 0.5).half()
    gam = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    bet = 0.05 * torch.randn(D, device="cuda", generator=g)
    lq = {}
    for name, lib in libs.items():
        q = torch.empty(R, D, dtype=torch.uint8, device="cuda")
        sc = torch.zeros(int(lib.miclip_mx_scale_bytes(R, D)), dtype=torch.uint8, device="cuda")
        assert lib.miclip_op_layernorm_mx(x.data_ptr(), 1, gam.data_ptr(), bet.data_ptr(), q.data_ptr(),
                                          sc.data_ptr(), R, D, s) == 0
        lq[name] = (q, sc)
    torch.cuda.synchronize()
    print(json.dumps({"check": "layernorm MX prev == new",
                      "equal": torch.equal(lq["prev"][0], lq["new"][0]) and torch.equal(lq["prev"][1], lq["new"][1])}),
          flush=True)
    res = {k: [] for k in ("attn_prev", "attn_new", "ln_prev", "ln_new")}
    o = torch.empty(B * N, W, device="cuda", dtype=torch.float16)
    for _ in range(4):
        for name, lib in libs.items():
            res["attn_" + name].append(round(timed(
                lambda: lib.miclip_op_attention(0, qkv.data_ptr(), o.data_ptr(), B, N, H, dh, 0, 0, s)), 4))
            q, sc = lq[name]
            res["ln_" + name].append(round(timed(
                lambda: lib.miclip_op_layernorm_mx(x.data_ptr(), 1, gam.data_ptr(), bet.data_ptr(),
                                                   q.data_ptr(), sc.data_ptr(), R, D, s)), 4))
    fl = 4.0 * B * H * N * N * dh
    for k, v in res.items():
        best = min(v)
        extra = {"tflops_best": round(fl / best / 1e9, 1)} if k.startswith("attn") else \
                {"gbs_best": round(R * D * 3.03 / best / 1e6, 1)}
        print(json.dumps({"op": k, "ms": v, **extra}), flush=True)


if __name__ == "__main__":
    main()
