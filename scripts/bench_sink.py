"""Does AsyncHostSink overlap the per-batch D2H with the encode?

Times compute_image_features over a host loader (CPU fp32 batches, as a
DataLoader yields them) three ways on one GPU:
  * device   : to_cpu=False (features stay on the GPU; the upper bound)
  * sink     : to_cpu=True  (miclip.feature_cache.AsyncHostSink: side-stream D2H
               into pinned memory, bounded depth)
  * sync     : the reference's loop shape, a synchronous `.to("cpu")` per batch
               (methods/utils.py:164, aihab_utils/feature_cache.py:131)
and prints one JSON line. Usage: python scripts/bench_sink.py [--model ViT-L/14]
[--batch 128] [--batches 16]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aihab-clip_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ViT-L/14")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import miclip
    from miclip.feature_cache import compute_image_features
    _, m, _ = miclip.load(a.model, device="cuda", compute_dtype="fp16", surface="openai")
    R = m.config.image_resolution
    g = torch.Generator().manual_seed(0)
    loader = [(torch.randn(a.batch, 3, R, R, generator=g), torch.arange(a.batch))
              for _ in range(a.batches)]
    m.reserve(a.batch)

    def sync_loop():
        feats = []
        for x, t in loader:
            feats.append(m.encode_image(x.cuda(non_blocking=True)).to("cpu"))
        return torch.cat(feats)

    ways = {"device": lambda: compute_image_features(m, loader, to_cpu=False),
            "sink": lambda: compute_image_features(m, loader, to_cpu=True),
            "sync": sync_loop}
    for f in ways.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in ways}
    for _ in range(a.rounds):
        for k, f in ways.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = f()
            if isinstance(out, tuple):
                out = out[0]
            if out.is_cuda:
                torch.cuda.synchronize()
            res[k].append(round(a.batch * a.batches / (time.perf_counter() - t0), 1))
    ref = compute_image_features(m, loader, to_cpu=False)[0].cpu()
    same = torch.equal(compute_image_features(m, loader, to_cpu=True)[0], ref)
    print(json.dumps({"what": "compute_image_features host-loader throughput (img/s)",
                      "model": a.model, "batch": a.batch, "batches": a.batches,
                      "img_per_s": res, "best": {k: max(v) for k, v in res.items()},
                      "sink_equals_device": same}), flush=True)


if __name__ == "__main__":
    main()
