"""Generate tests/golden/outliers.npz by running the REFERENCE outlier scorers on CPU.

Run in the build container only (needs /root/reference; the GPU box has none):

    PYTHONDONTWRITEBYTECODE=1 python oracle/make_golden_outliers.py

Inputs: a seeded synthetic embeddings cache -- 6 classes
of unequal size (12 .. 160 rows, so the heuristic k of compute_prototypes
spans 1 .. 4 modes), each a mixture of 1-3 unit-norm clusters in D = 96 plus
a few planted off-class rows -- with labels and a metadata frame shaped like
cache_openclip_embeddings' metadata.csv. A second, un-normalised copy
(random norms) exercises the re-normalisation branch of
_get_normalized_embeddings.

Outputs: the reference `SingleCentroidScorer.score_centroid_distance()` and
`MultiPrototypeScorer.score_prototype_distance()` frames
(tools/outlier_cleaning.py:295-383, 557-760) and their centroid/prototype
tensors, stored column by column. Nothing from the reference is copied: only
the numbers it produced.
"""
import importlib.util
import json
import os
import sys

import numpy as np
import pandas as pd
import torch

REF = os.environ.get("MICLIP_REFERENCE", "/root/reference")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.dont_write_bytecode = True
OUT = os.path.join(ROOT, "tests", "golden", "outliers.npz")

SIZES = [160, 12, 75, 130, 40, 20]
D = 96


def synthetic_cache(seed=0):
    g = np.random.default_rng(seed)
    embs, labels, names = [], [], []
    for c, n in enumerate(SIZES):
        modes = 1 + c % 3
        centers = g.normal(size=(modes, D))
        centers /= np.linalg.norm(centers, axis=1, keepdims=True)
        pick = g.integers(0, modes, n)
        x = centers[pick] + 0.35 * g.normal(size=(n, D)) / np.sqrt(D)
        off = g.choice(n, size=max(1, n // 25), replace=False)
        x[off] = g.normal(size=(len(off), D))          # planted off-class rows
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        embs.append(x)
        labels += [10 + 3 * c] * n                       # sparse label ids
        names += [f"img_{c}_{i:04d}.jpg" for i in range(n)]
    perm = g.permutation(len(labels))
    emb = np.concatenate(embs)[perm].astype(np.float32)
    lab = np.asarray(labels, np.int64)[perm]
    names = [names[i] for i in perm]
    meta = pd.DataFrame({"file_name": names, "ground_truth_num_label": lab,
                         "ground_truth_word_label": [f"class{v}" for v in lab],
                         "ground_truth_L2_num_label": lab % 4})
    scale = (0.5 + g.random(len(lab))).astype(np.float32)
    return emb, lab, meta, scale


def main():
    spec = importlib.util.spec_from_file_location(
        "_ref_outlier_cleaning", os.path.join(REF, "tools", "outlier_cleaning.py"))
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)

    emb, lab, meta, scale = synthetic_cache()
    out = {"emb": emb, "labels": lab, "scale": scale,
           "meta_file_name": np.asarray(meta["file_name"]).astype(str),
           "meta_word": np.asarray(meta["ground_truth_word_label"]).astype(str),
           "meta_l2": np.asarray(meta["ground_truth_L2_num_label"])}
    info = {}
    for tag, x in (("norm", emb), ("raw", emb * scale[:, None])):
        e = torch.from_numpy(np.ascontiguousarray(x))
        t = torch.from_numpy(lab)
        sc = ref.SingleCentroidScorer(e, t, meta)
        cent = sc.compute_centroids()
        df = sc.score_centroid_distance()
        keys = sorted(cent.centroids)
        out[f"{tag}_centroid_labels"] = np.asarray(keys)
        out[f"{tag}_centroids"] = torch.stack([cent.centroids[k] for k in keys]).numpy()
        for col in df.columns:
            v = np.asarray(df[col])
            out[f"{tag}_single_{col}"] = v.astype(str) if v.dtype == object else v
        mp = ref.MultiPrototypeScorer(e, t, meta)
        res = mp.compute_prototypes()
        dfm = mp.score_prototype_distance()
        out[f"{tag}_proto_k"] = np.asarray([res.k_per_class[k] for k in keys])
        out[f"{tag}_protos"] = torch.cat([res.prototypes[k].reshape(-1, D) for k in keys]).numpy()
        out[f"{tag}_proto_counts"] = np.concatenate(
            [np.asarray(res.prototype_counts[k]) for k in keys])
        for col in dfm.columns:
            v = np.asarray(dfm[col])
            out[f"{tag}_multi_{col}"] = v.astype(str) if v.dtype == object else v
        info[tag] = {"single_cols": list(df.columns), "multi_cols": list(dfm.columns)}
    out["meta"] = np.frombuffer(json.dumps(info).encode(), dtype=np.uint8)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
