"""Rank program of test_gpu_distributed.py::test_sharded_cache_gloo_world2_one_gpu (not a
test module): started by torch.distributed.run with two ranks that share cuda:0 over a
gloo group, each with its own HIP model (seeded weights, identical on both ranks): ViT-B/32,
ViT-L/14, ViT-L/14@336px (C2-C4) and open_clip ViT-H-14 in MX-fp8 (C5). Every
rank checks that the sharded encode and the sharded feature cache (both loader forms,
SURVEY §8e) equal its own single-process encode bit for bit, then prints RANK_OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aihab-clip_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    import miclip
    from miclip.feature_cache import (compute_image_features_sharded, shard_range,
                                      sharded_encode)
    from miclip.weights import synthetic_images
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == 2
    torch.cuda.set_device(0)
    for name, kw, res in (("ViT-B/32", {}, 224), ("ViT-L/14", {}, 224), ("ViT-L/14@336px", {}, 336),
                          ("ViT-H-14", {"compute_dtype": "mxfp8"}, 224)):
        check(miclip, name, kw, res, rank, world, compute_image_features_sharded, shard_range,
              sharded_encode, synthetic_images)
    dist.barrier()
    dist.destroy_process_group()
    print(f"RANK_OK {rank}", flush=True)


def check(miclip, name, kw, res, rank, world, compute_image_features_sharded, shard_range,
          sharded_encode, synthetic_images):
    """C2-C5's models (ViT-H-14 in MX-fp8, the stretch config)."""
    _, m, _ = miclip.load(name, device="cuda", **kw)
    n = 37
    imgs = torch.from_numpy(synthetic_images(n, res, seed=11))   # host batch, as a loader's
    ref = m.encode_image(imgs.cuda(), normalize=True)
    enc = lambda x: m.encode_image(x.cuda(), normalize=True)     # noqa: E731
    got = sharded_encode(enc, imgs, dim=ref.shape[1])
    assert got.device.type == "cuda" and torch.equal(got, ref), f"{name}: sharded_encode"
    # every rank walks the same loader, encodes its slice of each batch
    loader = [(imgs[i:i + 10], torch.arange(i, min(i + 10, n))) for i in range(0, n, 10)]
    feats, labels = compute_image_features_sharded(m, loader, normalize=True)
    assert torch.equal(feats, ref) and torch.equal(labels.cpu(), torch.arange(n)), f"{name}: same loader"
    # per-rank loader: only this rank's contiguous slice of each global batch of 16
    mine = []
    for b0 in range(0, n, 16):
        nb = min(16, n - b0)
        lo, hi = shard_range(nb, rank, world)
        mine.append((imgs[b0 + lo:b0 + hi], torch.arange(b0 + lo, b0 + hi)))
    feats, labels = compute_image_features_sharded(m, mine, normalize=True, per_rank=True)
    assert torch.equal(feats, ref) and torch.equal(labels.cpu(), torch.arange(n)), f"{name}: per-rank loader"
    print(f"rank {rank} {name}: ok", flush=True)
    del m
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
