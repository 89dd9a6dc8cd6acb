"""Outlier scoring of the embeddings cache vs the reference.

Golden: tests/golden/outliers.npz, produced by running the reference
tools/outlier_cleaning.py scorers on CPU (oracle/make_golden_outliers.py) on a
seeded synthetic cache, once already L2-normalised ("norm") and once with
random row norms ("raw", exercising the re-normalisation branch).

Bar (fp32): similarities / scores within 5e-6 absolute of the reference;
centroids / prototypes within 2e-6; integer columns (ranks, prototype ids,
sizes) exact except on rows whose reference score has a neighbour in its class
closer than 1e-5 (an order decided below fp32 noise). Rows are matched by
file_name (the frames are sorted by score, so near-ties may swap rows).
"""
import numpy as np
import pandas as pd
import pytest
import torch

from conftest import GOLDEN  # noqa: F401

TOL_SIM, TOL_VEC, TIE = 5e-6, 2e-6, 1e-5


@pytest.fixture(scope="module")
def fx():
    import os
    z = np.load(os.path.join(GOLDEN, "outliers.npz"))
    return {k: z[k] for k in z.files}


def _meta(fx):
    return pd.DataFrame({"file_name": fx["meta_file_name"],
                         "ground_truth_num_label": fx["labels"],
                         "ground_truth_word_label": fx["meta_word"],
                         "ground_truth_L2_num_label": fx["meta_l2"]})


def _golden_frame(fx, tag, kind, cols):
    return pd.DataFrame({c: fx[f"{tag}_{kind}_{c}"] for c in cols})


def _emb(fx, tag):
    e = fx["emb"] if tag == "norm" else fx["emb"] * fx["scale"][:, None]
    return torch.from_numpy(np.ascontiguousarray(e.astype(np.float32)))


# ---------------------------------------------------------------- CPU
def test_fixture_shapes(fx):
    n, d = fx["emb"].shape
    assert fx["labels"].shape == (n,) and d == 96
    assert fx["norm_single_outlier_score"].shape == (n,)
    assert int(fx["norm_proto_k"].sum()) == fx["norm_protos"].shape[0]


def test_validation_errors_before_device(fx):
    from miclip.outliers import SingleCentroidScorer, _validate_embeddings_labels
    e = _emb(fx, "norm")
    with pytest.raises(ValueError):
        _validate_embeddings_labels(e[:, :, None], torch.from_numpy(fx["labels"]))
    with pytest.raises(ValueError):
        SingleCentroidScorer(e[:10], torch.from_numpy(fx["labels"]), _meta(fx))
    with pytest.raises(TypeError):
        SingleCentroidScorer(e, torch.from_numpy(fx["labels"]), "not a frame")
    with pytest.raises(TypeError):
        _validate_embeddings_labels(e.to(torch.int32), torch.from_numpy(fx["labels"]))


def test_resolve_cache_paths(tmp_path):
    from miclip.outliers import resolve_cache_paths, load_cache
    p = resolve_cache_paths(tmp_path)
    assert p.embeddings.name == "embeddings.pt" and p.metadata.name == "metadata.csv"
    with pytest.raises(FileNotFoundError):
        load_cache(p)


# ---------------------------------------------------------------- GPU
def _near_tie_rows(g, score_col, group_cols):
    """file_names whose reference score has a same-group neighbour within TIE."""
    bad = set()
    for _, grp in g.groupby(group_cols):
        s = grp.sort_values(score_col)
        v = s[score_col].to_numpy()
        names = s["file_name"].to_numpy()
        close = np.zeros(len(v), bool)
        if len(v) > 1:
            d = np.diff(v) < TIE
            close[1:] |= d
            close[:-1] |= d
        bad |= set(names[close])
    return bad


def _compare(got, gold, float_cols, int_cols, rank_groups):
    m = gold.merge(got, on="file_name", suffixes=("_g", "_o"))
    assert len(m) == len(gold) == len(got)
    for c in float_cols:
        a, b = m[f"{c}_g"].to_numpy(np.float64), m[f"{c}_o"].to_numpy(np.float64)
        both_nan = np.isnan(a) & np.isnan(b)
        assert np.all(both_nan | (np.abs(a - b) <= TOL_SIM)), (c, np.nanmax(np.abs(a - b)))
    ties = set()
    for cols in rank_groups:
        ties |= _near_tie_rows(gold, "outlier_score", cols)
    keep = ~m["file_name"].isin(ties)
    for c in int_cols:
        a, b = m.loc[keep, f"{c}_g"].to_numpy(), m.loc[keep, f"{c}_o"].to_numpy()
        assert np.array_equal(a, b), (c, int((a != b).sum()))
    return int((~keep).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["norm", "raw"])
def test_single_centroid_matches_reference(fx, tag):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from miclip.outliers import SingleCentroidScorer
    sc = SingleCentroidScorer(_emb(fx, tag), torch.from_numpy(fx["labels"]), _meta(fx))
    cent = sc.compute_centroids()
    rows = torch.stack([cent.centroids[int(k)] for k in fx[f"{tag}_centroid_labels"]]).cpu().numpy()
    assert np.abs(rows - fx[f"{tag}_centroids"]).max() <= TOL_VEC
    df = sc.score_centroid_distance()
    cols = list(df.columns)
    gold = _golden_frame(fx, tag, "single", cols)
    _compare(df, gold, ["sim_to_centroid", "outlier_score", "pct_rank_in_class"],
             ["ground_truth_num_label", "class_size", "rank_in_class", "is_bottom_5pct"],
             [["ground_truth_num_label"]])


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["norm", "raw"])
def test_multi_prototype_matches_reference(fx, tag):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from miclip.outliers import MultiPrototypeScorer
    mp = MultiPrototypeScorer(_emb(fx, tag), torch.from_numpy(fx["labels"]), _meta(fx))
    res = mp.compute_prototypes()
    keys = sorted(res.prototypes)
    assert [res.k_per_class[k] for k in keys] == list(fx[f"{tag}_proto_k"])
    protos = torch.cat([res.prototypes[k].reshape(-1, 96) for k in keys]).cpu().numpy()
    assert np.abs(protos - fx[f"{tag}_protos"]).max() <= 1e-5
    df = mp.score_prototype_distance()
    cols = list(df.columns)
    gold = _golden_frame(fx, tag, "multi", cols)
    _compare(df, gold,
             ["sim_to_centroid", "outlier_score", "pct_rank_in_class", "sim_to_prototype",
              "pct_rank_in_prototype", "sim_to_other_class_best", "margin_to_other_class"],
             ["ground_truth_num_label", "class_size", "rank_in_class", "is_bottom_5pct",
              "prototype_id", "num_prototypes_in_class", "prototype_size", "rank_in_prototype"],
             [["ground_truth_num_label"], ["ground_truth_num_label", "prototype_id"]])


@pytest.mark.gpu
def test_class_sums_are_sequential_order_exact():
    """class_centroids sums rows in ascending sample order: bit-equal to a CPU index_add_."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from miclip.outliers import _class_centroids
    g = torch.Generator().manual_seed(3)
    x = torch.randn(5000, 768, generator=g)
    inv = torch.randint(0, 7, (5000,), generator=g)
    sums = torch.zeros(7, 768).index_add_(0, inv, x)
    counts = torch.bincount(inv, minlength=7)
    ref = torch.nn.functional.normalize(sums / counts[:, None].float(), dim=-1, eps=1e-12)
    cent, cnt = _class_centroids(x.cuda(), inv.numpy(), 7, 1e-12)
    assert np.array_equal(cnt, counts.numpy())
    assert (cent.cpu() - ref).abs().max().item() <= 1e-6


@pytest.mark.gpu
def test_proto_scores_large_vs_torch():
    """Many prototypes (several 64-wide tiles) and a ragged last sample tile."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from miclip.outliers import _proto_scores
    g = torch.Generator().manual_seed(5)
    N, P, D, K = 3001, 150, 1024, 37
    x = torch.nn.functional.normalize(torch.randn(N, D, generator=g), dim=-1)
    pr = torch.nn.functional.normalize(torch.randn(P, D, generator=g), dim=-1)
    owner = torch.randint(0, K, (P,), generator=g).to(torch.int32)
    cls = torch.randint(0, K, (N,), generator=g).to(torch.int32)
    own, arg, oth = _proto_scores(x.cuda(), pr.cuda(), owner.cuda(), cls.cuda())
    sim = (x.double() @ pr.double().t())
    same = cls[:, None].long() == owner[None, :].long()
    ref_own = sim.masked_fill(~same, -np.inf).max(1)
    ref_oth = sim.masked_fill(same, -np.inf).max(1).values
    has = same.any(1)
    assert torch.allclose(own.cpu().double()[has], ref_own.values[has], atol=1e-6)
    assert (own.cpu()[~has] == -np.inf).all()
    assert torch.allclose(oth.cpu().double(), ref_oth, atol=1e-6)
    # argmax agrees where the best own-class prototype is not a near tie
    top2 = sim.masked_fill(~same, -np.inf).topk(2, dim=1).values
    clear = has & ((top2[:, 0] - top2[:, 1]) > 1e-5)
    assert torch.equal(arg.cpu().long()[clear], ref_own.indices[clear])
