"""Probe: is the MX-fp8 encode deterministic at bs=512, and where do fp16-input rows differ?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "aihab-clip_amd"), ROOT]
import torch
import miclip
from miclip.weights import synthetic_images

name = sys.argv[1] if len(sys.argv) > 1 else "ViT-H-14"
dt = sys.argv[2] if len(sys.argv) > 2 else "mxfp8"
bs = int(sys.argv[3]) if len(sys.argv) > 3 else 512
_, m, _ = miclip.load(name, device="cuda", compute_dtype=dt, surface="openai")
x = torch.from_numpy(synthetic_images(bs, m.config.image_resolution, seed=77)).cuda()
runs = [m.encode_image(x).cpu() for _ in range(4)]
for i in range(1, 4):
    d = (runs[i] != runs[0]).any(1)
    print(f"fp32 run {i}: rows differing {d.sum().item()} {torch.nonzero(d).flatten()[:10].tolist()}")
h = m.encode_image(x.half()).cpu()
d = (h != runs[0]).any(1)
print(f"fp16 input: rows differing {d.sum().item()} {torch.nonzero(d).flatten()[:10].tolist()} max|d| {(h - runs[0]).abs().max().item():.3e}")
xr = x.half().float()
r = m.encode_image(xr).cpu()
d = (r != runs[0]).any(1)
print(f"fp32 of fp16-rounded input: rows differing {d.sum().item()}")
for s in (1,):
    m.set_splits(s)
    u = m.encode_image(x).cpu()
    d = (u != runs[0]).any(1)
    print(f"splits={s}: rows differing {d.sum().item()} {torch.nonzero(d).flatten()[:10].tolist()}")
