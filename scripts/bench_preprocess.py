#!/usr/bin/env python
"""Throughput of the on-device CLIP preprocessing kernel.

Workload: a batch of decoded uint8 RGB frames already in HBM (default 256 x
1080 x 1920, camera-trap video size) -> Resize(R, bicubic) + CenterCrop(R) +
ToTensor + Normalize -> float32 [B, 3, R, R]; R = 224 (ViT-L/14).
Timed with HIP events on torch's current stream (the stream the kernel runs on).

Roofline: HBM. Algorithmic bytes per image = the input rows x columns the
crop's bicubic taps touch (Resample.c bounds: center +- 2*scale) x 3 + the
float32 output 3*R*R*4; achieved = bytes / kernel time vs 8 TB/s.

CPU baseline: the reference's per-image transform (Pillow resize, the library
torchvision calls, + torchvision's crop / ToTensor / Normalize rules) on one
host core for a bounded sample.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "aihab-clip_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def window(in_size, out_size, lo, n):
    """Input index range [a, b) the outputs lo..lo+n-1 of a resize read."""
    scale = in_size / out_size
    support = 2.0 * max(scale, 1.0)
    a = max(int((lo + 0.5) * scale - support + 0.5), 0)
    b = min(int((lo + n - 0.5) * scale + support + 0.5), in_size)
    return a, b


def algorithmic_bytes(H, W, R):
    if W <= H:
        nw, nh = R, int(R * H / W)
    else:
        nw, nh = int(R * W / H), R
    top, left = int(round((nh - R) / 2.0)), int(round((nw - R) / 2.0))
    y0, y1 = window(H, nh, top, R)
    x0, x1 = window(W, nw, left, R)
    return (y1 - y0) * (x1 - x0) * 3 + 3 * R * R * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--model", default="ViT-L/14")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu-images", type=int, default=24)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import miclip
    from miclip.configs import MODEL_CONFIGS
    from miclip.weights import generate_state_dict
    cfg0 = MODEL_CONFIGS[args.model]
    # the kernel only needs the resolution; a 1-layer model of that resolution keeps setup fast
    from dataclasses import replace
    cfg = replace(cfg0, vision_layers=1, vision_width=256, transformer_width=256,
                  transformer_heads=4, transformer_layers=1, embed_dim=64)
    sd = {k: torch.from_numpy(v) for k, v in generate_state_dict(cfg, seed=0).items()}
    model = miclip.CLIP(cfg, sd, device="cuda")
    R, B, H, W = cfg.image_resolution, args.batch, args.height, args.width

    g = torch.Generator(device="cuda").manual_seed(0)
    # smooth-ish synthetic frames: low-frequency gradient + noise, uint8 HWC
    yy = torch.linspace(0, 6.28, H, device="cuda").view(1, H, 1, 1)
    xx = torch.linspace(0, 6.28, W, device="cuda").view(1, 1, W, 1)
    ph = torch.rand(B, 1, 1, 3, device="cuda", generator=g) * 6.28
    frames = (127 + 60 * torch.sin(xx * 3 + ph) * torch.cos(yy * 2 + ph)
              + torch.randn(B, H, W, 3, device="cuda", generator=g) * 20).clamp_(0, 255).to(torch.uint8)
    out = torch.empty(B, 3, R, R, device="cuda")
    for _ in range(3):
        model.preprocess_images(frames, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.iters):
        model.preprocess_images(frames, out=out)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.iters
    by = B * algorithmic_bytes(H, W, R)
    gbs = by / (ms * 1e-3) / 1e9

    cpu = None
    if not args.no_cpu_baseline:
        from oracle.pil_resample import transform_reference
        host = frames[: args.cpu_images].cpu().numpy()
        ok = np.array_equal(transform_reference(host[0], R), out[0].cpu().numpy())
        t0 = time.perf_counter()
        for i in range(host.shape[0]):
            transform_reference(host[i], R)
        dt = time.perf_counter() - t0
        cpu = {"value": round(host.shape[0] / dt, 2), "unit": "images/s", "cores": 1, "kind": "port",
               "sample": f"{host.shape[0]} frames {H}x{W} through Pillow {__import__('PIL').__version__} "
                         f"resize + torchvision crop/ToTensor/Normalize rules "
                         f"(oracle/pil_resample.transform_reference), one core, {dt:.1f}s; "
                         f"GPU output bit-identical on frame 0: {ok}"}
    line = {"metric": f"images/s preprocessed (uint8 {H}x{W}x3 -> CLIP float32 [3,{R},{R}])",
            "value": round(B / (ms * 1e-3), 1), "unit": "images/s", "ms_per_batch": round(ms, 4),
            "batch": B, "dtype": "u8->f32", "data": "synthetic",
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(gbs / 8000.0, 4), "traffic": None,
                         "algorithmic_bytes_per_image": algorithmic_bytes(H, W, R)},
            "cpu_baseline": cpu}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
