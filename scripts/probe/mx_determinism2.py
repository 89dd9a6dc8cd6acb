"""Probe: run-to-run determinism of a model's encode at a large batch, with the
batch split over 2 streams and unsplit (does the nondeterminism need both
streams?). Usage: mx_determinism2.py NAME DTYPE BS RUNS"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "aihab-clip_amd"), ROOT]
import torch
import miclip
from miclip.weights import synthetic_images

name, dt, bs, runs = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
_, m, _ = miclip.load(name, device="cuda", compute_dtype=dt, surface="openai")
x = torch.from_numpy(synthetic_images(bs, m.config.image_resolution, seed=77)).cuda()
for splits in (2, 1):
    m.set_splits(splits)
    ref = m.encode_image(x).cpu()
    bad = 0
    for i in range(runs):
        r = m.encode_image(x).cpu()
        d = (r != ref).any(1)
        if d.any():
            bad += 1
            print(f"  splits={splits} run {i}: rows {torch.nonzero(d).flatten()[:10].tolist()} max|d| {(r - ref).abs().max().item():.3e}", flush=True)
    print(f"{name} {dt} bs={bs} splits={splits}: {bad} of {runs} runs differ from the first", flush=True)
