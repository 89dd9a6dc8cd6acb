#!/usr/bin/env python
"""Eager vs HIP-graph-replayed encode_image at ViT-L/14 bs=256 (same process):
whether launch gaps between the ~170 kernels per stream cost anything."""
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
    _, m, _ = miclip.load("ViT-L/14", device="cuda", compute_dtype="fp16")
    m.reserve(B, 20)
    x = torch.from_numpy(synthetic_images(B, 224, seed=1)).cuda()
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
