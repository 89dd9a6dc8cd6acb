#!/usr/bin/env python
"""Bitwise comparison of GEMM variants against the default kernel (bench_ops
variant syntax, e.g. 259b) on the ViT-L/14 shapes: prints max |diff| per shape."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))
import torch  # noqa: E402
from miclip import _lib  # noqa: E402

SUFFIX = {"n": 1 << 16, "f": 1 << 17, "s": 1 << 18, "d": 1 << 19, "e": 1 << 20, "x": 1 << 21,
          "y": 1 << 22, "b": 1 << 23}


def parse(v):
    return int(v[:-1]) | SUFFIX[v[-1]] if v[-1] in SUFFIX else int(v)


def main():
    lib = _lib.load_library()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(1)
    M, W = int(os.environ.get("M", "32896")), 1024
    ok = True
    for name, N, K, epi, act in [("fc", 4 * W, W, 0, 1), ("proj", W, 4 * W, 4, 0)]:
        A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
        Wt = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).half()
        b = torch.randn(N, device="cuda", generator=g) * 0.1
        X0 = torch.randn(M, N, device="cuda", generator=g).half()
        outs = []
        for v in ["0"] + sys.argv[1:]:
            C = X0.clone() if epi == 4 else torch.empty(M, N, device="cuda", dtype=torch.float16)
            rc = lib.miclip_op_gemm(0, A.data_ptr(), Wt.data_ptr(), b.data_ptr(), C.data_ptr(), M, N, K,
                                    epi, act, parse(v), s)
            assert rc == 0, lib.miclip_last_error()
            outs.append((v, C))
        torch.cuda.synchronize()
        for v, C in outs[1:]:
            eq = torch.equal(C, outs[0][1])
            ok &= eq
            print(f"{name} variant {v}: bitwise {'equal' if eq else 'DIFFERENT'}, max|d| "
                  f"{(C.float() - outs[0][1].float()).abs().max().item():.3g}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
