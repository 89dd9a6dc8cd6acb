#!/usr/bin/env python
"""LayerNorm op timings (HIP events, torch's current stream) at the model shapes:
the MX-fp8-out kernel of C5 (ViT-H-14 bs=512), the fp16-in / bf16-out kernel of C2
(ViT-B/32 bs=256) and the fp16 kernel at ViT-L/14 bs=256 (ln_pre). One JSON line each.
MICLIP_LIB selects the library (same-box A/B)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    tag = os.path.basename(os.environ.get("MICLIP_LIB", "libmiclip.so"))
    for name, R, D in (("mx_c5", 512 * 257, 1280), ("bf16_c2", 256 * 50, 768), ("f16_l14", 256 * 257, 1024)):
        x = torch.randn(R, D, device="cuda", generator=g).half()
        gm = torch.rand(D, device="cuda", generator=g) + 0.5
        bt = torch.randn(D, device="cuda", generator=g) * 0.1
        if name.startswith("mx"):
            q = torch.empty(R, D, device="cuda", dtype=torch.uint8)
            sc = torch.empty(int(lib.miclip_mx_scale_bytes(R, D)), device="cuda", dtype=torch.uint8)

            def fn():
                assert lib.miclip_op_layernorm_mx(x.data_ptr(), 1, gm.data_ptr(), bt.data_ptr(), q.data_ptr(),
                                                  sc.data_ptr(), R, D, s) == 0
            by = R * D * 3
        else:
            code = 1 if name.startswith("bf16") else 0
            y = torch.empty(R, D, device="cuda", dtype=torch.bfloat16 if code else torch.float16)

            def fn():
                assert lib.miclip_op_layernorm(code, x.data_ptr(), gm.data_ptr(), bt.data_ptr(), y.data_ptr(),
                                               2, R, D, s) == 0
            by = R * D * 4
        ms = timeit(fn)
        print(json.dumps(dict(lib=tag, op=name, R=R, D=D, ms=round(ms, 4), gbs=round(by / ms / 1e6, 1))), flush=True)
    # the attention output's MX quantisation before C5's out-projection (quant_mx, fp16 in)
    R, D = 512 * 257, 1280
    x = torch.randn(R, D, device="cuda", generator=g).half()
    q = torch.empty(R, D, device="cuda", dtype=torch.uint8)
    sc = torch.empty(int(lib.miclip_mx_scale_bytes(R, D)), device="cuda", dtype=torch.uint8)

    def fq():
        assert lib.miclip_op_quant_mx(x.data_ptr(), 1, R, D, q.data_ptr(), sc.data_ptr(), s) == 0
    ms = timeit(fq)
    print(json.dumps(dict(lib=tag, op="quant_c5", R=R, D=D, ms=round(ms, 4), gbs=round(R * D * 3 / ms / 1e6, 1))),
          flush=True)


if __name__ == "__main__":
    main()
