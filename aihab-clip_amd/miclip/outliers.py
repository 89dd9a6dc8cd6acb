"""Outlier scoring of the embeddings cache on the GPU.

Counterpart of tools/outlier_cleaning.py (same names, arguments, outputs and
errors): `CachePaths`, `CentroidResult`, `MultiPrototypeResult`,
`resolve_cache_paths`, `load_cache`, `SingleCentroidScorer`,
`MultiPrototypeScorer`. The arithmetic on the embeddings runs in the HIP
kernels of csrc/scoring.hip through the C ABI:

  * row norms / re-normalisation      miclip_row_norms        (:229-247)
  * class centroids                   miclip_class_centroids  (:250-291)
  * cosine to own centroid            miclip_proto_scores     (:293-383)
  * nearest own-class prototype and
    best other-class prototype        miclip_proto_scores     (:557-760)

What stays on the host, as in the reference: label bookkeeping
(torch.unique), the spherical k-means fit of compute_prototypes (scikit-learn
KMeans with the reference's parameters, :488-498) and the pandas ranking /
quantile / sort post-processing. Embeddings live on the HIP device; there is
no CPU fallback.
"""
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import ctypes

import numpy as np
import pandas as pd
import torch

from . import _lib


@dataclass
class CachePaths:
    cache_dir: Path
    embeddings: Path
    labels: Path
    metadata: Path
    meta_json: Optional[Path] = None


@dataclass
class CentroidResult:
    centroids: Dict[int, torch.Tensor]
    class_counts: Dict[int, int]
    dim: int


@dataclass
class MultiPrototypeResult:
    prototypes: Dict[int, torch.Tensor]
    class_counts: Dict[int, int]
    prototype_counts: Dict[int, List[int]]
    k_per_class: Dict[int, int]
    dim: int


def resolve_cache_paths(cache_dir: Path) -> CachePaths:
    """embeddings.pt / labels.pt / metadata.csv / meta.json under cache_dir
    (the layout cache_openclip_embeddings writes)."""
    cache_dir = Path(cache_dir)
    return CachePaths(cache_dir=cache_dir, embeddings=cache_dir / "embeddings.pt",
                      labels=cache_dir / "labels.pt", metadata=cache_dir / "metadata.csv",
                      meta_json=cache_dir / "meta.json")


def _load_tensor_cpu(path: Path) -> torch.Tensor:
    """A cache file holds one tensor (loaded with weights_only=True)."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, torch.Tensor):
        return obj
    raise TypeError(f"Expected tensor at '{path}', got {type(obj).__name__}.")


def _validate_embeddings_labels(embeddings, labels, *, allow_empty=False):
    """Shape / dtype / row-count checks on an (embeddings [N, D], labels [N]) pair.

    Returns (embeddings, labels as int64 [N], N, D). The error types and texts
    are the reference's (tools/outlier_cleaning.py), since callers match on them.
    A [N, 1] label column is accepted as [N]."""
    if labels.ndim == 2 and labels.shape[-1] == 1:
        labels = labels[:, 0]
    checks = (
        (embeddings.ndim == 2, ValueError,
         lambda: f"Expected embeddings shape [N, D], got {tuple(embeddings.shape)}."),
        (labels.ndim == 1, ValueError,
         lambda: f"Expected labels shape [N], got {tuple(labels.shape)}."),
        (embeddings.is_floating_point(), TypeError,
         lambda: f"Expected floating embeddings, got dtype={embeddings.dtype}."),
    )
    for ok, exc, msg in checks:
        if not ok:
            raise exc(msg())
    n, d = (int(v) for v in embeddings.shape)
    if labels.shape[0] != n:
        raise ValueError(f"Row mismatch between embeddings and labels: {n} vs {int(labels.shape[0])}.")
    if n == 0 and not allow_empty:
        raise ValueError("Empty inputs: no samples available.")
    return embeddings, labels.long(), n, d


def load_cache(paths: CachePaths) -> Tuple[torch.Tensor, torch.Tensor, pd.DataFrame]:
    """(embeddings, labels, metadata) of a cache directory, rows cross-checked:
    the three files exist, embeddings / labels are a consistent pair, metadata.csv
    has one row per sample with file_name and ground_truth_num_label, and its labels
    equal labels.pt row for row (the first disagreeing row is reported)."""
    files = (paths.embeddings, paths.labels, paths.metadata)
    absent = [str(f) for f in files if not Path(f).is_file()]
    if absent:
        raise FileNotFoundError("Missing cache file(s): " + ", ".join(absent))
    embeddings, labels, n, _ = _validate_embeddings_labels(_load_tensor_cpu(paths.embeddings),
                                                           _load_tensor_cpu(paths.labels))
    metadata = pd.read_csv(paths.metadata)
    if len(metadata) != n:
        raise ValueError(f"Row mismatch between embeddings and metadata: {n} vs {len(metadata)}.")
    need = sorted({"file_name", "ground_truth_num_label"}.difference(metadata.columns))
    if need:
        raise ValueError(f"metadata.csv is missing required column(s): {', '.join(need)}")
    csv_labels = metadata["ground_truth_num_label"].astype(int).to_numpy()
    diff = np.flatnonzero(csv_labels != labels.numpy())
    if diff.size:
        i = int(diff[0])
        raise ValueError(f"Label mismatch between labels.pt and metadata.csv at row {i}: "
                         f"labels.pt={int(labels[i])}, metadata.csv={int(csv_labels[i])}.")
    return embeddings, labels, metadata


# ------------------------------------------------------------------ device ops
def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return _lib.stream_handle(dev)


def _row_norms(x: torch.Tensor, eps: float = 1e-12, normalize: bool = False):
    lib = _lib.load_library()
    norms = torch.empty(x.shape[0], device=x.device, dtype=torch.float32)
    out = torch.empty_like(x) if normalize else None
    with torch.cuda.device(x.device):
        _lib.check(lib.miclip_row_norms(_ptr(x), x.shape[0], x.shape[1], _ptr(norms), float(eps),
                                        _ptr(out), _stream(x.device)), "miclip_row_norms")
    return norms, out


def _class_centroids(x: torch.Tensor, inv: np.ndarray, K: int, eps: float):
    """normalize(per-class mean) with the rows of each class summed in sample order."""
    lib = _lib.load_library()
    order = np.argsort(inv, kind="stable").astype(np.int32)
    counts = np.bincount(inv, minlength=K)
    offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    dev = x.device
    order_d = torch.from_numpy(order).to(dev)
    off_d = torch.from_numpy(offsets).to(dev)
    D = x.shape[1]
    sums = torch.empty(K, D, device=dev, dtype=torch.float32)
    cent = torch.empty(K, D, device=dev, dtype=torch.float32)
    with torch.cuda.device(dev):
        _lib.check(lib.miclip_class_centroids(_ptr(x), _ptr(order_d), _ptr(off_d), K, D,
                                              float(eps), _ptr(sums), _ptr(cent), _stream(dev)),
                   "miclip_class_centroids")
    return cent, counts


def _proto_scores(x, protos, owner, cls, inv_nx=None, inv_np=None):
    lib = _lib.load_library()
    N, D = x.shape
    P = protos.shape[0]
    dev = x.device
    own = torch.empty(N, device=dev, dtype=torch.float32)
    arg = torch.empty(N, device=dev, dtype=torch.int32)
    oth = torch.empty(N, device=dev, dtype=torch.float32)
    with torch.cuda.device(dev):
        _lib.check(lib.miclip_proto_scores(_ptr(x), _ptr(protos), _ptr(owner), _ptr(cls),
                                           _ptr(inv_nx), _ptr(inv_np), N, P, D, _ptr(own),
                                           _ptr(arg), _ptr(oth), _stream(dev)),
                   "miclip_proto_scores")
    return own, arg, oth


def _device(device):
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError("miclip outlier scoring needs a HIP device (no CPU fallback)")
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


# ------------------------------------------------------------------ scorers
class SingleCentroidScorer:
    """Single-centroid scorer (tools/outlier_cleaning.py:178-383) on the GPU."""

    def __init__(self, embeddings: torch.Tensor, labels: torch.Tensor, metadata: pd.DataFrame,
                 *, normalize_tol: float = 1e-3, eps: float = 1e-12, device=None):
        embeddings, labels, num_samples, dim = _validate_embeddings_labels(
            embeddings, labels, allow_empty=False)
        if not isinstance(metadata, pd.DataFrame):
            raise TypeError(f"Expected metadata to be pandas DataFrame, got {type(metadata).__name__}.")
        if int(len(metadata)) != num_samples:
            raise ValueError("Row mismatch between embeddings and metadata: "
                             f"{num_samples} vs {int(len(metadata))}.")
        self.device = _device(device)
        self.embeddings = embeddings.detach().to(self.device, torch.float32).contiguous()
        self.labels = labels.detach().cpu()
        self.metadata = metadata.copy().reset_index(drop=True)
        self.num_samples = num_samples
        self.dim = dim
        self.normalize_tol = float(normalize_tol)
        self.eps = float(eps)
        self._centroids: Optional[CentroidResult] = None
        self._normalized_embeddings: Optional[torch.Tensor] = None
        if "ground_truth_num_label" in self.metadata.columns:
            meta_labels = torch.tensor(
                self.metadata["ground_truth_num_label"].astype(int).to_numpy(), dtype=torch.long)
            bad = torch.nonzero(meta_labels != self.labels, as_tuple=False).flatten()
            if int(bad.numel()) > 0:
                i = int(bad[0].item())
                raise ValueError("Label mismatch between labels tensor and metadata at row "
                                 f"{i}: labels={int(self.labels[i])}, metadata={int(meta_labels[i])}.")

    def _classes(self):
        uniq, inv = torch.unique(self.labels, sorted=True, return_inverse=True)
        return uniq, inv.numpy().astype(np.int64)

    def _get_normalized_embeddings(self) -> torch.Tensor:
        """Unit-norm rows on the device, computed once: the row norms come from the
        HIP kernel; rows are re-normalised (same kernel) only when some norm is off
        by more than normalize_tol; NaN / Inf norms are an error."""
        if self._normalized_embeddings is None:
            norms, _ = _row_norms(self.embeddings)
            if not torch.isfinite(norms).all().item():
                raise ValueError("Non-finite embedding norms found (NaN/Inf).")
            worst = (norms - 1.0).abs().max().item()
            emb = self.embeddings
            if worst > self.normalize_tol:
                print(f"[warn] Unnormalized embeddings detected (max |norm-1|={worst:.3e}); normalizing.")
                emb = _row_norms(self.embeddings, self.eps, normalize=True)[1]
            self._normalized_embeddings = emb
        return self._normalized_embeddings

    def compute_centroids(self, *, trim_frac: Optional[float] = None) -> CentroidResult:
        if trim_frac is not None:
            raise NotImplementedError("trim_frac is not implemented yet (planned follow-up).")
        if self._centroids is not None:
            return self._centroids
        emb = self._get_normalized_embeddings()
        uniq, inv = self._classes()
        K = int(uniq.numel())
        if K == 0:
            raise ValueError("No labels present to compute centroids.")
        cent, counts = _class_centroids(emb, inv, K, self.eps)
        self._centroids = CentroidResult(
            centroids={int(uniq[i]): cent[i] for i in range(K)},
            class_counts={int(uniq[i]): int(counts[i]) for i in range(K)}, dim=self.dim)
        return self._centroids

    def _frame(self):
        scores = self.metadata.copy().reset_index(drop=True)
        scores["ground_truth_num_label"] = self.labels.numpy().astype(int)
        if "ground_truth_word_label" not in scores.columns:
            scores["ground_truth_word_label"] = ""
        if "ground_truth_L2_num_label" not in scores.columns:
            scores["ground_truth_L2_num_label"] = -1
        if "file_name" not in scores.columns:
            scores["file_name"] = ""
        return scores

    @staticmethod
    def _class_ranks(scores, sim_col, counts):
        scores["class_size"] = scores["ground_truth_num_label"].map(counts).astype(int)
        scores["rank_in_class"] = (scores.groupby("ground_truth_num_label")["outlier_score"]
                                   .rank(method="first", ascending=False).astype(int))
        scores["pct_rank_in_class"] = scores["rank_in_class"] / scores["class_size"]
        p05 = scores.groupby("ground_truth_num_label")[sim_col].transform(
            lambda col: col.quantile(0.05))
        scores["is_bottom_5pct"] = scores[sim_col] <= p05

    def score_centroid_distance(self, *, centroids: Optional[CentroidResult] = None) -> pd.DataFrame:
        res = centroids if centroids is not None else (
            self._centroids if self._centroids is not None else self.compute_centroids())
        if int(res.dim) != self.dim:
            raise ValueError(f"Centroid dim mismatch: expected {self.dim}, got {int(res.dim)}.")
        emb = self.embeddings
        if not bool(torch.isfinite(emb).all()):
            raise ValueError("Non-finite embeddings found (NaN/Inf).")
        uniq, inv = self._classes()
        missing = [int(v) for v in uniq if int(v) not in res.centroids]
        if missing:
            raise ValueError("Missing centroid(s) for label(s): " + ", ".join(str(v) for v in sorted(missing)))
        rows = torch.stack([res.centroids[int(v)].reshape(-1) for v in uniq]).to(
            self.device, torch.float32).contiguous()
        if not bool(torch.isfinite(rows).all()):
            raise ValueError("Non-finite centroid values found (NaN/Inf).")
        K = rows.shape[0]
        # cosine_similarity(emb, centroid[inv]): x/max(|x|,eps) . c/max(|c|,eps)
        nx, _ = _row_norms(emb)
        nc, _ = _row_norms(rows)
        inv_nx = 1.0 / nx.clamp_min(self.eps)
        inv_nc = 1.0 / nc.clamp_min(self.eps)
        owner = torch.arange(K, device=self.device, dtype=torch.int32)
        cls = torch.from_numpy(inv.astype(np.int32)).to(self.device)
        sim, _, _ = _proto_scores(emb, rows, owner, cls, inv_nx, inv_nc)
        sim = sim.cpu().numpy()
        scores = self._frame()
        scores["sim_to_centroid"] = sim
        scores["outlier_score"] = 1.0 - sim
        self._class_ranks(scores, "sim_to_centroid", res.class_counts)
        cols = ["file_name", "ground_truth_num_label", "ground_truth_word_label",
                "ground_truth_L2_num_label", "sim_to_centroid", "outlier_score", "class_size",
                "rank_in_class", "pct_rank_in_class", "is_bottom_5pct"]
        return scores[cols].sort_values(by=["outlier_score", "ground_truth_num_label", "file_name"],
                                        ascending=[False, True, True]).reset_index(drop=True)


class MultiPrototypeScorer(SingleCentroidScorer):
    """Multi-prototype scorer (tools/outlier_cleaning.py:386-760) on the GPU."""

    def __init__(self, embeddings, labels, metadata, *, normalize_tol: float = 1e-3,
                 eps: float = 1e-12, device=None):
        super().__init__(embeddings, labels, metadata, normalize_tol=normalize_tol, eps=eps,
                         device=device)
        self._prototypes: Optional[MultiPrototypeResult] = None
        self._prototype_config = None

    def compute_prototypes(self, *, k_mode: str = "heuristic", k_fixed: int = 2, k_max: int = 4,
                           min_samples_per_proto: int = 15, random_state: int = 0,
                           n_init: int = 10, max_iter: int = 100) -> MultiPrototypeResult:
        if k_mode not in {"heuristic", "fixed"}:
            raise ValueError(f"Unsupported k_mode '{k_mode}'. Expected one of: heuristic, fixed.")
        for name, v in (("k_fixed", k_fixed), ("k_max", k_max),
                        ("min_samples_per_proto", min_samples_per_proto), ("n_init", n_init),
                        ("max_iter", max_iter)):
            if int(v) < 1:
                raise ValueError(f"{name} must be >= 1, got {v}.")
        config = (str(k_mode), int(k_fixed), int(k_max), int(min_samples_per_proto),
                  int(random_state), int(n_init), int(max_iter))
        if self._prototypes is not None and self._prototype_config == config:
            return self._prototypes
        try:
            from sklearn.cluster import KMeans
        except ImportError as exc:
            raise ImportError("scikit-learn is required for multi-prototype scoring. "
                              "Install it to use MultiPrototypeScorer.") from exc
        emb = self._get_normalized_embeddings()
        uniq, inv = self._classes()
        if int(uniq.numel()) == 0:
            raise ValueError("No labels present to compute prototypes.")
        K = int(uniq.numel())
        means, counts = _class_centroids(emb, inv, K, self.eps)   # the k = 1 prototypes
        prototypes, class_counts, prototype_counts, k_per_class = {}, {}, {}, {}
        for ci in range(K):
            label_id = int(uniq[ci])
            n_c = int(counts[ci])
            class_counts[label_id] = n_c
            if k_mode == "heuristic":
                base_k = 1 if n_c < 20 else 3 if n_c < 100 else 4 if n_c < 200 else \
                    5 if n_c < 300 else 6
            else:
                base_k = int(k_fixed)
            base_k = min(base_k, int(k_max))
            k_c = max(1, int(min(base_k, n_c, max(1, n_c // int(min_samples_per_proto)))))
            if k_c == 1:
                center = means[ci:ci + 1]
                if not bool(torch.isfinite(center).all()):
                    raise ValueError(f"Non-finite prototype found for class {label_id} (k=1).")
                prototypes[label_id] = center
                prototype_counts[label_id] = [n_c]
                k_per_class[label_id] = 1
                continue
            idx = torch.from_numpy(np.nonzero(inv == ci)[0]).to(self.device)
            x_c = emb.index_select(0, idx).contiguous()
            km = KMeans(n_clusters=k_c, random_state=int(random_state), n_init=int(n_init),
                        max_iter=int(max_iter))
            km.fit(x_c.cpu().numpy())
            centers = torch.from_numpy(km.cluster_centers_.astype(np.float32)).to(self.device)
            _, centers = _row_norms(centers.contiguous(), self.eps, normalize=True)
            if not bool(torch.isfinite(centers).all()):
                raise ValueError(f"Non-finite prototype centers found for class {label_id}.")
            # re-assign by cosine (x_c @ centers^T, argmax) for the prototype counts
            zeros = torch.zeros(k_c, device=self.device, dtype=torch.int32)
            zc = torch.zeros(x_c.shape[0], device=self.device, dtype=torch.int32)
            _, arg, _ = _proto_scores(x_c, centers, zeros, zc)
            cnt = np.bincount(arg.cpu().numpy(), minlength=k_c)
            prototypes[label_id] = centers
            prototype_counts[label_id] = [int(v) for v in cnt]
            k_per_class[label_id] = k_c
        self._prototypes = MultiPrototypeResult(prototypes=prototypes, class_counts=class_counts,
                                                prototype_counts=prototype_counts,
                                                k_per_class=k_per_class, dim=self.dim)
        self._prototype_config = config
        return self._prototypes

    def score_prototype_distance(self, *, prototypes: Optional[MultiPrototypeResult] = None) -> pd.DataFrame:
        res = prototypes if prototypes is not None else (
            self._prototypes if self._prototypes is not None else self.compute_prototypes())
        if int(res.dim) != self.dim:
            raise ValueError(f"Prototype dim mismatch: expected {self.dim}, got {int(res.dim)}.")
        emb = self._get_normalized_embeddings()
        uniq, inv = self._classes()
        missing = [int(v) for v in uniq if int(v) not in res.prototypes]
        if missing:
            raise ValueError("Missing prototype(s) for label(s): " + ", ".join(str(v) for v in sorted(missing)))
        # all prototypes in sorted label order (the reference's all_prototypes)
        blocks, owners, first, sizes = [], [], {}, []
        label_to_ci = {int(v): i for i, v in enumerate(uniq)}
        for label_id in sorted(res.prototypes.keys()):
            block = res.prototypes[label_id]
            block = (block.unsqueeze(0) if block.ndim == 1 else block).to(self.device, torch.float32)
            if int(block.shape[1]) != self.dim:
                raise ValueError(f"Prototype dim mismatch in class {label_id}: "
                                 f"expected {self.dim}, got {int(block.shape[1])}.")
            if not bool(torch.isfinite(block).all()):
                raise ValueError(f"Non-finite prototype values found for class {label_id}.")
            counts_c = res.prototype_counts[label_id]
            if len(counts_c) != int(block.shape[0]):
                raise ValueError(f"prototype_counts length mismatch for class {label_id}: "
                                 f"{len(counts_c)} vs {int(block.shape[0])}.")
            first[label_id] = sum(b.shape[0] for b in blocks)
            blocks.append(block)
            owners += [label_to_ci.get(label_id, -1)] * int(block.shape[0])
            sizes += list(counts_c)
        protos = torch.cat(blocks).contiguous()
        owner = torch.tensor(owners, device=self.device, dtype=torch.int32)
        cls = torch.from_numpy(inv.astype(np.int32)).to(self.device)
        own, arg, oth = _proto_scores(emb, protos, owner, cls)
        own, arg, oth = own.cpu().numpy(), arg.cpu().numpy(), oth.cpu().numpy()
        lab = self.labels.numpy().astype(int)
        first_of = np.asarray([first[int(v)] for v in lab])
        proto_id = arg - first_of
        n_in_class = np.asarray([res.prototypes[int(v)].reshape(-1, self.dim).shape[0] for v in lab])
        proto_size = np.asarray(sizes)[arg]
        if int(uniq.numel()) <= 1:
            oth = np.full_like(own, np.nan)
            margin = np.full_like(own, np.nan)
        else:
            oth = np.where(np.isinf(oth), np.nan, oth).astype(np.float32)
            margin = own - oth
        scores = self._frame()
        scores["method"] = "multi_prototype"
        scores["sim_to_prototype"] = own
        scores["sim_to_centroid"] = scores["sim_to_prototype"]
        scores["outlier_score"] = 1.0 - own
        scores["prototype_id"] = proto_id.astype(int)
        scores["num_prototypes_in_class"] = n_in_class.astype(int)
        scores["prototype_size"] = proto_size.astype(int)
        self._class_ranks(scores, "sim_to_prototype", res.class_counts)
        scores["rank_in_prototype"] = (scores.groupby(["ground_truth_num_label", "prototype_id"])
                                       ["outlier_score"].rank(method="first", ascending=False)
                                       .astype(int))
        scores["pct_rank_in_prototype"] = scores["rank_in_prototype"] / scores["prototype_size"]
        scores["sim_to_other_class_best"] = oth
        scores["margin_to_other_class"] = margin
        cols = ["file_name", "ground_truth_num_label", "ground_truth_word_label",
                "ground_truth_L2_num_label", "sim_to_centroid", "outlier_score", "class_size",
                "rank_in_class", "pct_rank_in_class", "is_bottom_5pct", "method",
                "sim_to_prototype", "prototype_id", "num_prototypes_in_class", "prototype_size",
                "rank_in_prototype", "pct_rank_in_prototype", "sim_to_other_class_best",
                "margin_to_other_class"]
        return scores[cols].sort_values(by=["outlier_score", "ground_truth_num_label", "file_name"],
                                        ascending=[False, True, True]).reset_index(drop=True)
