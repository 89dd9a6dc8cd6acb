"""The reference's batched-encode drivers, run on the HIP model.

Each counterpart in miclip.feature_cache / miclip.classifier is driven the way
the reference drives its own, and its outputs are checked against the reference
goldens (tests/golden, made by running clip/model.py): values, row order, dtype
and the on-disk layout the reference writes.

  clip_classifier                utils.py:31-57
  compute_image_features         methods/utils.py:142-173
  compute_image_features_test    methods/utils.py:175-189 (+ ProLIP VisProjViT, methods/ProLIP.py:31-41)
  cache_openclip_embeddings      aihab_utils/feature_cache.py:98-186
  cache_preprojection_features   aihab_utils/feature_cache.py:189-250
  AsyncHostSink                  SURVEY §8f row 2 (the async replacement of `.to('cpu')` per batch)
  miclip.load(<checkpoint path>) clip/clip.py:117-137 + build_model clip/model.py:396-433
"""
import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3


def _one_minus_cos(a, b, dim=-1):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return (1 - torch.nn.functional.cosine_similarity(a, b, dim=dim)).numpy()


_models = {}


def _model(name):
    import miclip
    if name not in _models:
        _models.clear()
        torch.cuda.empty_cache()
        _models[name] = miclip.load(name, device="cuda", compute_dtype="fp16")[1]
    return _models[name]


@pytest.fixture(scope="module", autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    yield
    _models.clear()


def _golden_tokenizer(g):
    """clip.tokenize for exactly the golden prompts (the BPE vocabulary is not on
    the GPU box): prompt string -> its reference-tokenised row."""
    table = {p: torch.from_numpy(g["tokens"][i]).long() for i, p in enumerate(g["meta"]["prompts"])}
    return lambda texts: torch.stack([table[t] for t in texts])


def _loader(imgs, labels, bs, meta=None):
    out = []
    for i in range(0, len(imgs), bs):
        b = (torch.from_numpy(imgs[i:i + bs]), torch.from_numpy(labels[i:i + bs]))
        if meta is not None:
            b = b + ({k: v[i:i + bs] for k, v in meta.items()},)
        out.append(b)
    return out


@pytest.mark.parametrize("tag,name,template", [("vitb32", "ViT-B/32", "a habitat photo of {}."),
                                               ("vitl14", "ViT-L/14", "{}")])
def test_clip_classifier_matches_golden(golden, tag, name, template):
    from miclip.classifier import clip_classifier
    g = golden(tag)
    prompts = g["meta"]["prompts"]
    if template == "{}":
        classnames = list(prompts)
    else:
        pre, post = template.split("{}")
        classnames = [p[len(pre):len(p) - len(post)] for p in prompts]
    m = _model(name)
    texts, before, weights = clip_classifier(classnames, [template], m, tokenize=_golden_tokenizer(g))
    C = len(prompts)
    assert weights.shape == (m.config.embed_dim, C) and weights.device.type == "cuda"
    assert before.shape == (1, C, m.config.transformer_width)
    assert torch.equal(texts.cpu(), torch.from_numpy(g["tokens"]).long())
    d = _one_minus_cos(weights.cpu().t(), g["text_weights"].T)
    print(f"{tag}: clip_classifier text_weights 1-cos max {d.max():.2e}")
    assert d.max() <= COS_TOL
    assert torch.allclose(weights.norm(dim=0), torch.ones(C, device="cuda"), atol=1e-5)
    db = _one_minus_cos(before[0].cpu(), g["text_before"])
    assert db.max() <= COS_TOL


def test_compute_image_features_row_order(golden):
    """Golden images through a loader in batches of 3 (ragged last batch)."""
    from miclip.feature_cache import compute_image_features
    from miclip.weights import synthetic_images
    g = golden("vitb32")
    n = g["meta"]["n_images"]
    imgs = synthetic_images(n, 224, seed=0)
    labels = np.arange(100, 100 + n, dtype=np.int64)[::-1].copy()
    m = _model("ViT-B/32")
    f_cpu, l_cpu = compute_image_features(m, _loader(imgs, labels, 3), to_cpu=True)
    assert f_cpu.device.type == "cpu" and f_cpu.dtype == torch.float32 and f_cpu.shape == (n, 768)
    assert torch.equal(l_cpu, torch.from_numpy(labels))
    d = _one_minus_cos(f_cpu, g["image"])
    print(f"compute_image_features 1-cos max {d.max():.2e}")
    assert d.max() <= COS_TOL
    f_dev, l_dev = compute_image_features(m, _loader(imgs, labels, 3), to_cpu=False)
    assert f_dev.device.type == "cuda" and l_dev.device.type == "cuda"
    assert torch.equal(f_dev.cpu(), f_cpu) and torch.equal(l_dev.cpu(), l_cpu)
    # batch size does not change a row (batch-invariant kernels)
    f_one, _ = compute_image_features(m, _loader(imgs, labels, n), to_cpu=True)
    assert torch.equal(f_one, f_cpu)


def test_compute_image_features_test_with_projector(golden):
    """ProLIP eval: callable projector (VisProjViT: x @ visual.proj), then the head;
    accuracy against labels = the golden top-1 (rows whose margin is safe) is 100 %."""
    from miclip.feature_cache import compute_image_features, compute_image_features_test
    from miclip.weights import synthetic_images
    g = golden("vitb32")
    n = g["meta"]["n_images"]
    imgs = synthetic_images(n, 224, seed=0)
    m = _model("ViT-B/32")
    vit_proj = m.state_dict()["visual.proj"]

    class VisProjViT(torch.nn.Module):          # methods/ProLIP.py:31-41
        def __init__(self, p):
            super().__init__()
            self.vit_proj = torch.nn.Parameter(p.clone())

        def forward(self, x):
            return x @ self.vit_proj

    tw = torch.from_numpy(g["text_weights"]).cuda()
    top1 = g["topk"][:, 0]
    sure = g["margins"] > 0.05
    acc_callable = compute_image_features_test(m, _loader(imgs[sure], top1[sure], 3), VisProjViT(vit_proj), tw)
    acc_matrix = compute_image_features_test(m, _loader(imgs[sure], top1[sure], 3), vit_proj, tw)
    assert acc_callable == 100.0 and acc_matrix == 100.0
    # ProLIP.py:286-293 verbatim on top of compute_image_features
    feats, labels = compute_image_features(m, _loader(imgs, g["topk"][:, 0], 4))
    logits = 100. * torch.nn.functional.normalize(VisProjViT(vit_proj)(feats), dim=-1) @ tw
    assert (logits - torch.from_numpy(g["logits"]).cuda()).abs().max().item() < 0.5
    agree = (logits.argmax(1).cpu().numpy() == g["topk"][:, 0])
    assert agree[sure].all()


def test_cache_openclip_embeddings_layout(golden, tmp_path):
    """embeddings.pt / labels.pt / metadata.csv / meta.json exactly as the reference writes them."""
    import pandas as pd
    from miclip.feature_cache import cache_openclip_embeddings
    from miclip.weights import synthetic_images
    g = golden("vitb32")
    n = g["meta"]["n_images"]
    imgs = synthetic_images(n, 224, seed=0)
    labels = np.resize(np.array([3, 1, 4, 1, 5, 9, 2, 6], dtype=np.int64), n)
    meta = {"file_name": [f"img_{i:03d}.jpg" for i in range(n)],
            "plot_word_label": [f"class{l}" for l in labels],
            "l2_label": torch.arange(n) % 3}
    cfg = {"root_path": str(tmp_path), "dataset": "cs", "seed": 1, "clip_backend": "openai",
           "backbone": "ViT-B/32",
           "finetune": {"cache_embeddings_dir": "feat_cache_vis", "cache_embeddings_normalize": True}}
    m = _model("ViT-B/32")
    d = cache_openclip_embeddings(cfg, m, _loader(imgs, labels, 3, meta), split="Test",
                                  checkpoint_path="ckpt.pt")
    assert d == tmp_path / "feat_cache_vis" / "ViTB32_cs" / "test" / "seed1"
    emb = torch.load(d / "embeddings.pt", weights_only=True)
    lab = torch.load(d / "labels.pt", weights_only=True)
    assert emb.dtype == torch.float32 and emb.shape == (n, 768)
    assert torch.allclose(emb.norm(dim=1), torch.ones(n), atol=1e-5)
    ref = torch.nn.functional.normalize(torch.from_numpy(g["image"]), dim=-1)
    assert _one_minus_cos(emb, ref).max() <= COS_TOL
    assert torch.equal(lab, torch.from_numpy(labels))
    df = pd.read_csv(d / "metadata.csv")
    assert list(df.columns) == ["file_name", "ground_truth_num_label", "ground_truth_word_label",
                                "ground_truth_L2_num_label"]
    assert df["file_name"].tolist() == meta["file_name"]
    assert df["ground_truth_num_label"].tolist() == labels.tolist()
    assert df["ground_truth_word_label"].tolist() == meta["plot_word_label"]
    assert df["ground_truth_L2_num_label"].tolist() == (np.arange(n) % 3).tolist()
    info = json.loads((d / "meta.json").read_text())
    assert set(info) == {"timestamp", "split", "normalized", "num_samples", "dim",
                         "checkpoint_path", "cache_dir"}
    assert info["split"] == "Test" and info["normalized"] is True and info["num_samples"] == n
    assert info["dim"] == 768 and info["checkpoint_path"] == "ckpt.pt" and info["cache_dir"] == str(d)
    # 2-tuples: default metadata; unnormalised; bad batches raise like the reference
    cfg["finetune"]["cache_embeddings_normalize"] = False
    d2 = cache_openclip_embeddings(cfg, m, _loader(imgs, labels, 4), split="val")
    raw = torch.load(d2 / "embeddings.pt", weights_only=True)
    assert _one_minus_cos(raw, g["image"]).max() <= COS_TOL
    assert not torch.allclose(raw.norm(dim=1), torch.ones(n), atol=1e-3)
    df2 = pd.read_csv(d2 / "metadata.csv", keep_default_na=False)
    assert df2["file_name"].tolist() == [""] * n and df2["ground_truth_L2_num_label"].tolist() == [-1] * n
    with pytest.raises(ValueError, match="Expected batch"):
        cache_openclip_embeddings(cfg, m, [(torch.from_numpy(imgs[:2]),)], split="bad")


def test_cache_preprojection_features_layout(golden, tmp_path):
    from miclip.feature_cache import (_feature_cache_exists, cache_preprojection_features,
                                      compute_image_features)
    from miclip.weights import synthetic_images
    g = golden("vitb32")
    n = g["meta"]["n_images"]
    imgs = synthetic_images(n, 224, seed=0)
    labels = np.arange(n, dtype=np.int64) % 5
    cfg = {"root_path": str(tmp_path), "dataset": "cs", "seed": 2, "shots": 16,
           "backbone": "ViT-B/32", "aug_views": 2}
    m = _model("ViT-B/32")
    d = cache_preprojection_features(cfg, {"clip_model": m}, _loader(imgs, labels, 3), {"train_size": n})
    assert d == tmp_path / "features_ViTB32_cs" / "16_shot" / "seed2"
    assert _feature_cache_exists(d, 2) and not _feature_cache_exists(d, 3)
    f0 = torch.load(d / "f0.pth", weights_only=True)
    f1 = torch.load(d / "f1.pth", weights_only=True)
    lab = torch.load(d / "label.pth", weights_only=True)
    # fp16 like the reference's fp16 model writes them: the fp32 features rounded once
    assert f0.dtype == torch.float16 and f0.shape == (n, 768)
    assert _one_minus_cos(f0.float(), g["image"]).max() <= COS_TOL   # pre-projection, not normalised
    assert torch.equal(f0, f1) and torch.equal(lab, torch.from_numpy(labels))
    f32, _ = compute_image_features(m, _loader(imgs, labels, 3), to_cpu=True)
    assert torch.equal(f0, f32.half())
    cfg32 = dict(cfg, cache_dtype="fp32", root_path=str(tmp_path / "f32"))
    d32 = cache_preprojection_features(cfg32, {"clip_model": m}, _loader(imgs, labels, 3), None)
    assert torch.equal(torch.load(d32 / "f0.pth", weights_only=True), f32)
    with pytest.raises(ValueError):
        cache_preprojection_features(dict(cfg, cache_dtype="int8"), {"clip_model": m},
                                     _loader(imgs, labels, 3), None)


@pytest.mark.parametrize("proj,norm", [(False, False), (True, True), (False, True)])
def test_encode_image_out_dtype(golden, proj, norm):
    """out_dtype fp16 / bf16: the fp32 features rounded once (RNE) in the head's
    launch sequence -- bit for bit the fp32 result's .to(dtype), all paths."""
    from miclip.weights import synthetic_images
    g = golden("vitb32")
    imgs = torch.from_numpy(synthetic_images(g["meta"]["n_images"], 224, seed=0)).cuda()
    m = _model("ViT-B/32")
    f32 = m.encode_image(imgs, normalize=norm, apply_proj=proj)
    for dt in (torch.float16, torch.bfloat16):
        h = m.encode_image(imgs, normalize=norm, apply_proj=proj, out_dtype=dt)
        assert h.dtype == dt and torch.equal(h, f32.to(dt))
        out = torch.empty_like(h)
        assert m.encode_image(imgs, normalize=norm, apply_proj=proj, out=out) is out
        assert torch.equal(out, h)
    with pytest.raises(ValueError):
        m.encode_image(imgs, out_dtype=torch.int8)


def test_async_host_sink_depth_below_batches():
    """More batches than the in-flight depth: the sink waits for old copies, keeps
    push order, and the result equals the synchronous per-batch .to('cpu')."""
    from miclip.feature_cache import AsyncHostSink
    g = torch.Generator(device="cuda").manual_seed(0)
    sink = AsyncHostSink(depth=2)
    ref = []
    for i in range(9):
        x = torch.randn(5 + i, 64, device="cuda", generator=g) * (i + 1)
        y = x * 2 + 1                       # produced on the current stream just before the push
        sink.push(y)
        ref.append(y.to("cpu"))
        del x, y                            # the sink keeps its own reference alive
        assert len(sink._pending) <= 2
    out = sink.result()
    assert out.device.type == "cpu" and torch.equal(out, torch.cat(ref))
    cpu = AsyncHostSink(depth=1)
    cpu.push(torch.ones(2, 3))
    cpu.push(torch.zeros(1, 3))
    assert torch.equal(cpu.result(), torch.cat([torch.ones(2, 3), torch.zeros(1, 3)]))


def test_load_checkpoint_path_roundtrip(tmp_path):
    """miclip.load(<state-dict file>) (clip/clip.py:117-137): shapes inferred like
    build_model, same encode as the name-resolved model, bit for bit."""
    import miclip
    from miclip.weights import synthetic_images
    m = _model("ViT-B/32")
    path = tmp_path / "vitb32_seed0.pt"
    torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, path)
    sd, m2, pre = miclip.load(str(path), device="cuda")
    assert m2.config == m.config and set(sd) == set(m.state_dict())
    x = torch.from_numpy(synthetic_images(5, 224, seed=9)).cuda()
    assert torch.equal(m2.encode_image(x), m.encode_image(x))
    tok = torch.zeros(2, 77, dtype=torch.long)
    tok[:, 0], tok[0, 1:4], tok[0, 4], tok[1, 1], tok[1, 2] = 49406, torch.tensor([320, 1125, 539]), 49407, 786, 49407
    a, b = m.encode_text(tok.cuda()), m2.encode_text(tok.cuda())
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    # a {"state_dict": ...} wrapper and extra keys build_model drops are accepted
    torch.save({"state_dict": {**{k: v.detach().cpu() for k, v in m.state_dict().items()},
                               "input_resolution": torch.tensor(224)}}, tmp_path / "wrapped.pt")
    _, m3, _ = miclip.load(str(tmp_path / "wrapped.pt"), device="cuda")
    assert torch.equal(m3.encode_image(x), m.encode_image(x))
    with pytest.raises(RuntimeError, match="not found"):
        miclip.load(str(tmp_path / "missing.pt"), device="cuda")
    del m2, m3


def test_weight_load_paths_agree():
    """miclip_model_load_weights (host fp32, one staging upload + device cast) and
    miclip_model_load_weights_device (the Parameters themselves) build the same
    handle; refresh_weights re-uploads an in-place edit device to device."""
    from miclip.model import _DTYPES, _Handle
    from miclip.weights import synthetic_images
    m = _model("ViT-B/32")
    x = torch.from_numpy(synthetic_images(3, 224, seed=1)).cuda()
    ref = m.encode_image(x)
    h = _Handle(m.config, _DTYPES["fp16"][0], 0)
    h.load([(k, v.detach().float().cpu().numpy()) for k, v in m.state_dict().items()])
    saved = m._handle
    try:
        m._handle = h
        assert torch.equal(m.encode_image(x), ref)
    finally:
        m._handle = saved
        h.close()
    keep = m.visual.ln_post.bias.detach().clone()
    with torch.no_grad():
        m.visual.ln_post.bias.add_(0.5)
    m.refresh_weights()
    moved = m.encode_image(x)
    assert not torch.equal(moved, ref)
    with torch.no_grad():
        m.visual.ln_post.bias.copy_(keep)
    m.refresh_weights()
    assert torch.equal(m.encode_image(x), ref)
