"""Parity metrics shared by the GPU parity tests (test infrastructure).

`one_minus_cos` is the north star's per-row embedding metric. `centred_one_minus_cos`
removes each set's mean feature first: CLIP features of different images share a
large common component (random-init towers even more so), so the raw 1-cos can be
small for a kernel that mixed up images; the centred form compares only the
image-specific parts, where two different images are ~orthogonal (1-cos ~ 1).
Both sets must hold the same images in the same order.
"""
import numpy as np
import torch


def one_minus_cos(a, b, dim=-1):
    a = torch.as_tensor(a, dtype=torch.float64).cpu()
    b = torch.as_tensor(b, dtype=torch.float64).cpu()
    return (1 - torch.nn.functional.cosine_similarity(a, b, dim=dim)).numpy()


def centred_one_minus_cos(a, b):
    a = torch.as_tensor(a, dtype=torch.float64).cpu()
    b = torch.as_tensor(b, dtype=torch.float64).cpu()
    assert a.shape == b.shape and a.shape[0] >= 2
    return one_minus_cos(a - a.mean(0), b - b.mean(0))


def separation(feats):
    """Smallest 1-cos between the features of two DIFFERENT images of a set."""
    f = torch.nn.functional.normalize(torch.as_tensor(feats, dtype=torch.float64), dim=-1)
    n = f.shape[0]
    off = (1 - f @ f.T)[~torch.eye(n, dtype=torch.bool)]
    return float(off.min())


def report(tag, feats, ref, tol, centred_tol):
    """Asserts the raw and centred per-row bounds; prints them beside the golden
    set's own inter-image separation (how far apart two different images are)."""
    d = one_minus_cos(feats, ref)
    dc = centred_one_minus_cos(feats, ref)
    sep = separation(ref)
    print(f"{tag}: image 1-cos max {d.max():.2e} (tol {tol:.0e}), centred {dc.max():.2e} "
          f"(tol {centred_tol:.0e}); golden inter-image 1-cos min {sep:.2e} "
          f"= {sep / tol:.0f}x tol over {len(ref)} images")
    assert d.max() <= tol, f"{tag}: 1-cos {d.max():.3e} > {tol}"
    assert dc.max() <= centred_tol, f"{tag}: centred 1-cos {dc.max():.3e} > {centred_tol}"
    return d, dc


def top1_report(tag, top1, golden_top1, sure, min_rows=None):
    """Top-1 agreement on the rows whose golden margin clears the measured logit
    error; the golden top-1 column must hold >= 3 distinct classes, so a kernel that
    returned one feature for every image could not pass."""
    distinct = len(set(np.asarray(golden_top1).tolist()))
    agree = np.asarray(top1) == np.asarray(golden_top1)
    print(f"{tag}: top-1 agree {agree.sum()}/{len(agree)}, asserted on {int(sure.sum())} rows, "
          f"{distinct} distinct golden classes")
    assert distinct >= 3, f"{tag}: golden top-1 has only {distinct} classes"
    min_rows = len(agree) // 2 if min_rows is None else min_rows
    assert int(sure.sum()) >= min_rows, f"{tag}: too few rows clear the margin"
    assert np.all(agree[sure])
