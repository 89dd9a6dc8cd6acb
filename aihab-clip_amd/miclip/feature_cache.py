"""Batched-encode drivers of the reference, on the HIP encode path.

Counterparts (same names, arguments, outputs, file layout and error behaviour):
  * compute_image_features        methods/utils.py:142-173
  * compute_image_features_test   methods/utils.py:175-189
  * cache_openclip_embeddings     aihab_utils/feature_cache.py:98-186
  * cache_preprojection_features  aihab_utils/feature_cache.py:189-250
  * _feature_cache_dir / _embedding_cache_dir / _canonical_backbone_name /
    _feature_cache_exists          aihab_utils/feature_cache.py:18-65, 253-261

plus what the reference does not have:
  * AsyncHostSink: in-order asynchronous D2H of each batch into pinned host
    memory on a side stream instead of a synchronous
    `.to("cpu")` per batch;
  * prepare_images: loaders may yield decoded uint8 images, transformed on
    the GPU by `CLIP.preprocess_images`;
and the multi-GPU variant:
  * shard_range / sharded_encode / compute_image_features_sharded: each rank
    encodes a contiguous slice of the image batch and the L2-normalised (or
    raw) embeddings are all-gathered over RCCL (torch.distributed backend
    "nccl" on ROCm) back into the single-GPU row order, so cached
    embeddings.pt rows still line up with labels.pt / metadata.csv;
  * ShardedBatchLoader / gather_shards (per_rank=True): each rank reads and
    decodes only its own slice of every global batch.

Differences that matter to callers: compute_image_features returns fp32 by
default (the reference's GPU path returns the fp16 model's dtype; pass
out_dtype=torch.float16 for that); the pre-projection cache f{v}.pth is fp16 as
the reference writes it (cfg "cache_dtype": "fp16" default, "fp32" / "bf16");
the encode itself runs in the C ABI, with the optional normalise and the output
rounding fused into its head.
"""
import json
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F


def _canonical_backbone_name(backbone: str) -> str:
    if not backbone:
        return "unknown"
    if backbone == "ViT-B/16":
        return "ViTB16"
    if backbone == "ViT-B/32":
        return "ViTB32"
    name = backbone.replace("hf-hub:", "hf-hub_")
    return name.replace("/", "_").replace(" ", "_").replace(":", "_")


def _backbone(cfg) -> str:
    backend = str(cfg.get("clip_backend", "openai")).lower()
    if backend == "openclip":
        return cfg.get("open_clip_model", cfg.get("backbone", "RN50"))
    return cfg.get("backbone", "RN50")


def _feature_cache_dir(cfg) -> Path:
    root = Path(cfg.get("root_path", "./"))
    shots = int(cfg.get("shots", 0) or 0)
    seed = int(cfg.get("seed", 1) or 1)
    return (root / f"features_{_canonical_backbone_name(_backbone(cfg))}_{cfg.get('dataset', 'cs')}"
            / f"{shots}_shot" / f"seed{seed}")


def _embedding_cache_dir(cfg, split: str) -> Path:
    root = Path(cfg.get("root_path", "./"))
    ft = cfg.get("finetune", {}) or {}
    out_root = Path(ft.get("cache_embeddings_dir", "feat_cache_vis"))
    if not out_root.is_absolute():
        out_root = root / out_root
    seed = int(cfg.get("seed", 1) or 1)
    return (out_root / f"{_canonical_backbone_name(_backbone(cfg))}_{cfg.get('dataset', 'cs')}"
            / str(split).lower() / f"seed{seed}")


def _feature_cache_exists(cache_dir: Path, aug_views: int) -> bool:
    cache_dir = Path(cache_dir)
    if not cache_dir.exists() or not (cache_dir / "label.pth").is_file():
        return False
    return all((cache_dir / f"f{v}.pth").is_file() for v in range(aug_views))


_CACHE_DTYPES = {"fp16": torch.float16, "float16": torch.float16, "half": torch.float16,
                 "fp32": torch.float32, "float32": torch.float32, "float": torch.float32,
                 "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


def _cache_dtype(name, default: str) -> torch.dtype:
    if name is None:
        name = default
    if isinstance(name, torch.dtype):
        return name
    try:
        return _CACHE_DTYPES[str(name).lower()]
    except KeyError:
        raise ValueError(f"unknown cache dtype {name!r} (fp16, fp32 or bf16)") from None


def _encode(clip_model, images, out_dtype=None, **kw):
    """encode_image with the output element type fused into the HIP head where the
    model is a miclip model; other models' features are cast."""
    if out_dtype is None:
        return clip_model.encode_image(images, **kw)
    if hasattr(clip_model, "zero_shot"):
        return clip_model.encode_image(images, out_dtype=out_dtype, **kw)
    return clip_model.encode_image(images, **kw).to(out_dtype)


def _model_device(clip_model):
    try:
        params = list(clip_model.parameters())
        return params[0].device if params else torch.device("cuda")
    except Exception:
        return torch.device("cuda")


class AsyncHostSink:
    """In-order device -> host copies that never stall the encode loop.

    The reference moves every batch to the host with a synchronous
    `.to("cpu")` (methods/utils.py:164, aihab_utils/feature_cache.py:131),
    which drains the GPU once per batch. Here each pushed device tensor is
    copied on a side HIP stream (ordered after the producing stream by a
    stream wait) into pinned host memory; at most `depth` copies are in flight
    (older ones are waited for, so device memory held by pending copies stays
    bounded). `result()` waits for the tail and concatenates in push order.
    CPU tensors pass straight through.
    """

    def __init__(self, depth: int = 4):
        self.depth = max(1, int(depth))
        self._pending = []
        self._parts = []
        self._stream = None

    def push(self, t: torch.Tensor) -> None:
        t = t.detach()
        if not t.is_cuda:
            self._parts.append(t)
            return
        if self._stream is None:
            self._stream = torch.cuda.Stream(t.device)
        cur = torch.cuda.current_stream(t.device)
        self._stream.wait_stream(cur)
        host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        with torch.cuda.stream(self._stream):
            host.copy_(t, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        t.record_stream(self._stream)
        self._pending.append(ev)
        self._parts.append(host)
        while len(self._pending) > self.depth:
            self._pending.pop(0).synchronize()

    def result(self) -> torch.Tensor:
        for ev in self._pending:
            ev.synchronize()
        self._pending.clear()
        return torch.cat(self._parts, dim=0) if self._parts else torch.empty(0)


def is_raw_batch(images) -> bool:
    """True for decoded uint8 images (list of HxWxC arrays/tensors or a uint8 [B,H,W,C])."""
    if isinstance(images, torch.Tensor):
        return images.dtype == torch.uint8 and images.dim() == 4
    return isinstance(images, (list, tuple)) and len(images) > 0 and \
        getattr(images[0], "dtype", None) in (np.uint8, torch.uint8)


def prepare_images(model, images, device):
    """Model-ready float32 [B,3,R,R] on `device`: decoded uint8 batches go through the
    on-device transform (`CLIP.preprocess_images`); tensors that
    the loader already transformed (the reference's path) are moved as they are."""
    if is_raw_batch(images):
        if not hasattr(model, "preprocess_images"):
            raise ValueError("uint8 image batches need a miclip model (on-device preprocessing)")
        return model.preprocess_images(images)
    return images.to(device, non_blocking=True)


@torch.no_grad()
def compute_image_features(clip_model, loader, to_cpu: bool = False, out_dtype=None):
    """Pre-projection features and labels of every batch (methods/utils.py:142-173).

    With to_cpu the per-batch host copies are asynchronous (AsyncHostSink);
    loaders may also yield decoded uint8 images (prepare_images). out_dtype
    (torch.float16 / bfloat16) rounds the features in the encode's own head
    launch sequence (fp32 by default)."""
    device = _model_device(clip_model)
    feats, labels = ([], []) if not to_cpu else (AsyncHostSink(), [])
    for images, target in loader:
        x = _encode(clip_model, prepare_images(clip_model, images, device), out_dtype)
        if to_cpu:
            feats.push(x)
            labels.append(target.detach().to("cpu"))
        else:
            feats.append(x)
            labels.append(target.to(device, non_blocking=True))
    feats = feats.result() if to_cpu else torch.cat(feats, dim=0)
    return feats, torch.cat(labels, dim=0)


@torch.no_grad()
def compute_image_features_test(clip_model, loader, proj, text_weights):
    """Top-1 accuracy (%) of the zero-shot head (methods/utils.py:175-189).

    `proj` is the [Wv, E] projection matrix or a callable such as ProLIP's
    VisProjViT; normalise -> 100 * f @ W -> argmax runs in the HIP head kernel."""
    device = _model_device(clip_model)
    hits = []
    for images, target in loader:
        x = clip_model.encode_image(prepare_images(clip_model, images, device))
        f = proj(x) if callable(proj) and not isinstance(proj, torch.Tensor) else x @ proj.to(x)
        _, top = clip_model.zero_shot(f, text_weights, 100.0, k=1, apply_proj=False)
        hits += (top[:, 0].cpu() == target.cpu()).tolist()
    return 100 * float(np.mean(hits))


def _to_py(v: Any) -> Any:
    if isinstance(v, torch.Tensor):
        return v.item() if v.numel() == 1 else v.detach().cpu().tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


def _metadata_rows(metadata: Any, batch_size: int) -> List[Dict[str, Any]]:
    if not isinstance(metadata, dict):
        print("[warn] metadata missing; writing default values in metadata.csv."
              if metadata is None else
              "[warn] metadata is not a dict; writing default values in metadata.csv.")
        return [{} for _ in range(batch_size)]
    return [{k: _to_py(v[i] if isinstance(v, (list, tuple, np.ndarray, torch.Tensor)) else v)
             for k, v in metadata.items()} for i in range(batch_size)]


@torch.no_grad()
def cache_openclip_embeddings(cfg: dict, model, loader, split: str = "test",
                              checkpoint_path: Optional[str] = None) -> Path:
    """embeddings.pt / labels.pt / metadata.csv / meta.json (aihab_utils/feature_cache.py:98-186)."""
    import pandas as pd
    ft = cfg.get("finetune", {}) or {}
    normalize = bool(ft.get("cache_embeddings_normalize", True))
    # open_clip's model is fp32 in the reference (embeddings.pt fp32)
    out_dtype = _cache_dtype(ft.get("cache_embeddings_dtype"), "fp32")
    cache_dir = _embedding_cache_dir(cfg, split)
    cache_dir.mkdir(parents=True, exist_ok=True)
    device = _model_device(model)
    model.eval()
    sink, labels_list, rows = AsyncHostSink(), [], []
    for batch in loader:
        if isinstance(batch, (list, tuple)) and len(batch) == 3:
            images, targets, metadata = batch
        elif isinstance(batch, (list, tuple)) and len(batch) == 2:
            images, targets = batch
            metadata = None
        else:
            raise ValueError("Expected batch to be (images, targets) or (images, targets, metadata).")
        images = prepare_images(model, images, device)
        if hasattr(model, "zero_shot"):          # miclip model: normalise fused into ln_post
            feats = model.encode_image(images, normalize=normalize, out_dtype=out_dtype)
        else:
            feats = model.encode_image(images)
            if normalize:
                feats = F.normalize(feats, dim=-1)
            feats = feats.to(out_dtype)
        sink.push(feats)
        t = targets.detach().to("cpu")
        labels_list.append(t)
        for i, row in enumerate(_metadata_rows(metadata, int(t.shape[0]))):
            rows.append({"file_name": row.get("file_name", ""),
                         "ground_truth_num_label": int(t[i].item()),
                         "ground_truth_word_label": row.get("plot_word_label", ""),
                         "ground_truth_L2_num_label": row.get("l2_label", -1)})
    feats_all = sink.result()
    labels_all = torch.cat(labels_list, dim=0)
    torch.save(feats_all, cache_dir / "embeddings.pt")
    torch.save(labels_all, cache_dir / "labels.pt")
    cols = ["file_name", "ground_truth_num_label", "ground_truth_word_label",
            "ground_truth_L2_num_label"]
    pd.DataFrame(rows).reindex(columns=cols).to_csv(cache_dir / "metadata.csv", index=False)
    info = {"timestamp": datetime.now().strftime("%Y-%m-%d %H:%M:%S"), "split": str(split),
            "normalized": normalize, "num_samples": int(feats_all.shape[0]),
            "dim": int(feats_all.shape[1]) if feats_all.ndim == 2 else None,
            "checkpoint_path": str(checkpoint_path) if checkpoint_path is not None else None,
            "cache_dir": str(cache_dir)}
    with (cache_dir / "meta.json").open("w") as f:
        json.dump(info, f, indent=2)
    return cache_dir


@torch.no_grad()
def cache_preprojection_features(cfg, clip_bundle: dict, dl_tr, info: dict):
    """f{v}.pth per augmentation view + label.pth (aihab_utils/feature_cache.py:189-250).

    The features are fp16 like the reference's (its clip.load(..., device="cuda")
    model is fp16, so compute_image_features returns fp16, :211); cfg
    "cache_dtype" "fp32" / "bf16" picks another element type."""
    clip_model = clip_bundle["clip_model"]
    cache_dir = _feature_cache_dir(cfg)
    num_views = int(cfg.get("aug_views", 1) or 1)
    out_dtype = _cache_dtype(cfg.get("cache_dtype"), "fp16")
    expected_n = info.get("train_size") if info else None
    if expected_n is None and hasattr(dl_tr, "dataset"):
        expected_n = len(dl_tr.dataset)
    clip_model.eval()
    for v in range(num_views):
        feats_t, labels_t = compute_image_features(clip_model, dl_tr, to_cpu=True,
                                                   out_dtype=out_dtype)
        fpath = cache_dir / f"f{v}.pth"
        fpath.parent.mkdir(parents=True, exist_ok=True)
        torch.save(feats_t, fpath)
        if v == 0:
            torch.save(labels_t, cache_dir / "label.pth")
        loaded = torch.load(fpath, map_location="cpu", weights_only=True)
        print({"view": v, "features.dtype": str(feats_t.dtype),
               "reload_shape_ok": tuple(loaded.shape) == tuple(feats_t.shape),
               "rows_match_labels": feats_t.shape[0] == labels_t.shape[0],
               "rows_match_expected": expected_n is None or feats_t.shape[0] == int(expected_n)})
    return cache_dir


# ---------------------------------------------------------------- multi-GPU --

def shard_range(n: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of n items for `rank` (first n % world ranks get one more)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


@torch.no_grad()
def sharded_encode(encode_fn, images, group=None, dim: Optional[int] = None):
    """Encode this rank's contiguous slice of `images` and all-gather the rows.

    `images` is the full batch (every rank sees the same batch, e.g. from a
    deterministic loader) -- only rows shard_range(n, rank, world) are encoded
    here. Shards are padded to equal length for all_gather_into_tensor and the
    result is trimmed back, so the output equals encode_fn(images) row for row
    (the row order aihab_utils/feature_cache.py:144-162 relies on).

    The collective's buffers live where the backend needs them, whatever device
    the loader's images are on: nccl (RCCL) -> this rank's current HIP device,
    gloo -> host. A rank whose shard is empty (n < world) still joins the
    gather; it needs `dim`. Without an initialised process group this is
    encode_fn(images).
    """
    if not (dist.is_available() and dist.is_initialized()):
        return encode_fn(images)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = images.shape[0] if isinstance(images, torch.Tensor) else len(images)
    lo, hi = shard_range(n, rank, world)
    local = encode_fn(images[lo:hi]) if hi > lo else None
    width = dim if dim is not None else (local.shape[1] if local is not None else None)
    if width is None:
        raise ValueError("sharded_encode needs `dim` when a rank has an empty shard")
    dev = _collective_device(group)
    per = -(-n // world)
    if (local is not None and hi - lo == per and local.device == dev
            and local.dtype == torch.float32 and local.is_contiguous()):
        buf = local
    else:
        buf = torch.zeros(per, width, device=dev, dtype=torch.float32)
        if local is not None:
            buf[: hi - lo] = local
    out = torch.empty(world * per, width, device=dev, dtype=torch.float32)
    dist.all_gather_into_tensor(out, buf, group=group)
    if n != world * per:
        out = torch.cat([out[r * per: r * per + (shard_range(n, r, world)[1] - shard_range(n, r, world)[0])]
                         for r in range(world)])
    return out if local is None else out.to(local.device)


def _collective_device(group):
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


@torch.no_grad()
def gather_shards(local, group=None, width: Optional[int] = None, dtype=torch.float32,
                  counts: Optional[List[int]] = None):
    """All-gather per-rank row blocks of possibly different lengths, in rank order.

    For loaders that hand each rank only its own contiguous slice of a global
    batch (ShardedBatchLoader): the ranks exchange their row counts (one tiny
    all-gather), pad to the longest, all-gather, and drop the padding, so the
    result is the global batch in its original order when rank r holds the r-th
    slice. `local` may be None (an empty shard); then `width` (columns, 0 for a
    1-D block such as labels) is required. `counts` (every rank's row count, when
    the caller knows them, e.g. shard_range of a known batch) skips the count
    exchange and the host sync its result needs. Without a process group: `local`."""
    if not (dist.is_available() and dist.is_initialized()):
        return local
    world = dist.get_world_size(group)
    dev = _collective_device(group)
    n_local = 0 if local is None else int(local.shape[0])
    if local is not None:
        width = int(local.shape[1]) if local.dim() == 2 else 0
        dtype = local.dtype
    if width is None:
        raise ValueError("gather_shards needs `width` when a rank has an empty shard")
    if counts is None:
        counts = torch.empty(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(counts, torch.tensor([n_local], dtype=torch.int64, device=dev),
                                    group=group)
        counts = counts.tolist()
    elif len(counts) != world or counts[dist.get_rank(group)] != n_local:
        raise ValueError(f"counts {counts} do not match this rank's {n_local} rows / world {world}")
    counts = [int(c) for c in counts]
    per = max(counts)
    shape = (per, width) if width else (per,)
    buf = torch.zeros(shape, dtype=dtype, device=dev)
    if n_local:
        buf[:n_local] = local.to(dev)
    out = torch.empty((world * per,) + shape[1:], dtype=dtype, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = torch.cat([out[r * per: r * per + c] for r, c in enumerate(counts)])
    return out if local is None else out.to(local.device)


class ShardedBatchLoader:
    """Per-rank loader: global batch b covers dataset items [b*bs, min(n, (b+1)*bs));
    this rank reads and decodes only its contiguous slice shard_range(len, rank,
    world) of it, so no rank touches the other ranks' images (the reference's
    DataLoader, aihab_utils/feature_cache.py:114-142, decodes the whole batch).
    Yields (images, targets) from `collate_fn` over (image, target) items, or
    (None, empty targets) when the slice is empty (a last batch smaller than the
    world). compute_image_features_sharded(..., per_rank=True) restores the
    global order with gather_shards."""

    def __init__(self, dataset, batch_size: int, rank: Optional[int] = None,
                 world: Optional[int] = None, collate_fn=None):
        self.dataset = dataset
        self.batch_size = int(batch_size)
        init = dist.is_available() and dist.is_initialized()
        self.rank = rank if rank is not None else (dist.get_rank() if init else 0)
        self.world = world if world is not None else (dist.get_world_size() if init else 1)
        self.collate_fn = collate_fn or self._stack

    @staticmethod
    def _stack(items):
        imgs = [i[0] if isinstance(i[0], torch.Tensor) else torch.as_tensor(i[0]) for i in items]
        return torch.stack(imgs), torch.as_tensor([int(i[1]) for i in items], dtype=torch.int64)

    def __len__(self):
        return -(-len(self.dataset) // self.batch_size)

    def __iter__(self):
        n = len(self.dataset)
        for b0 in range(0, n, self.batch_size):
            nb = min(self.batch_size, n - b0)
            lo, hi = shard_range(nb, self.rank, self.world)
            if hi > lo:
                yield self.collate_fn([self.dataset[b0 + i] for i in range(lo, hi)])
            else:
                yield None, torch.empty(0, dtype=torch.int64)


@torch.no_grad()
def compute_image_features_sharded(clip_model, loader, normalize: bool = True, group=None,
                                   per_rank: bool = False):
    """compute_image_features over an image-batch-sharded node; returns (features,
    labels) on the rank's device in the single-GPU row order.

    per_rank=False: every rank walks the same loader, encodes its slice of each
    batch (sharded_encode) and receives the all-gathered (normalised) embeddings.
    per_rank=True: the loader yields only this rank's slice of each global batch
    (ShardedBatchLoader: each rank reads and decodes only its own images); the
    features and the labels are gathered back into global order (gather_shards)."""
    device = _model_device(clip_model)
    dim = getattr(clip_model, "image_dim", None) or clip_model.config.vision_width

    def enc(x):
        return clip_model.encode_image(prepare_images(clip_model, x, device), normalize=normalize)
    feats, labels = [], []
    for images, target in loader:
        if per_rank:
            local = enc(images) if images is not None and len(images) else None
            feats.append(gather_shards(local, group=group, width=dim).to(device))
            labels.append(gather_shards(target.to(torch.int64), group=group, width=0).to(device))
        else:
            feats.append(sharded_encode(enc, images, group=group, dim=dim))
            labels.append(target.to(device))
    return torch.cat(feats), torch.cat(labels)
