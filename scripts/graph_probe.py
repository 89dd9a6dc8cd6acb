#!/usr/bin/env python
"""Eager vs HIP-graph-replayed encode_image (same process): whether launch gaps
between the kernels cost anything.  graph_probe.py [B] [model] [dtype]
(default 256 ViT-L/14 fp16; C2: 256 ViT-B/32 bf16)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))

import torch  # noqa: E402

import miclip  # noqa: E402
from miclip.weights import synthetic_images  # noqa: E402


def timed(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    name = sys.argv[2] if len(sys.argv) > 2 else "ViT-L/14"
    dtype = sys.argv[3] if len(sys.argv) > 3 else "fp16"
    _, m, _ = miclip.load(name, device="cuda", compute_dtype=dtype)
    m.reserve(B, 20)
    R = m.config.image_resolution
    x = torch.from_numpy(synthetic_images(B, R, seed=1)).cuda()
    eager_out = m.encode_image(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            m.encode_image(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = m.encode_image(x)
    g.replay()
    torch.cuda.synchronize()
    print("graph output equals eager:", bool(torch.equal(out, eager_out)))
    for r in range(3):
        te = timed(lambda: m.encode_image(x), 10)
        tg = timed(g.replay, 10)
        print(f"round {r}: eager {te * 1e3:.3f} ms ({B / te:.0f} img/s)  graph {tg * 1e3:.3f} ms ({B / tg:.0f} img/s)")


if __name__ == "__main__":
    main()
