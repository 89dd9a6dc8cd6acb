"""CPU oracle: fp32 torch-CPU restatement of the reference CLIP encode path.

TEST INFRASTRUCTURE ONLY. Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module; the product path
(`aihab-clip_amd/miclip`) never does, and fails loudly when its HIP library
is missing instead of falling back here.

What it restates (all citations relative to the reference checkout):
  * `VisionTransformer.forward`          clip/model.py:216-235 (pre-projection output)
  * `ResidualAttentionBlock.forward`     clip/model.py:183-186
  * `LayerNorm` (fp32 compute)           clip/model.py:151-157
  * `QuickGELU`                          clip/model.py:160-162
  * `nn.MultiheadAttention` slow path    torch/nn/functional.py multi_head_attention_forward
    (packed in-proj -> per-head SDPA -> out-proj), batch_first=False
  * `CLIP.encode_text` (tuple output)    clip/model.py:338-353, causal mask 323-329
  * `clip_classifier`                    utils.py:31-57
  * zero-shot head                       methods/ProLIP.py:38-41, 288-293
  * cosine cache normalise               aihab_utils/feature_cache.py:126-127

It runs in the reference's CPU precision (fp32: clip/clip.py:135-136) and in
the reference's LND layout, using the same torch ops in the same order, so it
is bit-exact with the imported reference module on the same inputs
(checked by `oracle/make_golden.py` and pinned by `tests/golden/*.npz`).

ViT-H-14 (open_clip shapes): the same graph with exact GELU
and 80-wide vision heads. open_clip itself is absent from the container and
unpinned by the reference (configs/base.yaml names models, not a version), so
this config is pinned against the reference's own clip/model.py modules with
those two substitutions (`make_golden.py` vith14) -- "parity unpinned" with
respect to open_clip's code.

Parity pinning: the reference has no tests or golden vectors of its own
(SURVEY §4). The goldens under tests/golden/ were produced by importing the
reference `clip/model.py` in the build container and running it on the
seeded weights/inputs of `miclip.weights`; `make_golden.py` is the script.
"""
import torch
import torch.nn.functional as F


def _t(sd, name):
    v = sd[name]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(v)


def layer_norm(x, w, b):
    # clip/model.py:154-157 -- upcast to fp32, nn.LayerNorm (eps=1e-5), cast back
    orig = x.dtype
    return F.layer_norm(x.float(), (x.shape[-1],), w, b, 1e-5).type(orig)


def quick_gelu(x):
    # clip/model.py:160-162
    return x * torch.sigmoid(1.702 * x)


def gelu_erf(x):
    # nn.GELU() (approximate='none'): the MLP activation of open_clip's
    # ResidualAttentionBlock (act_layer default; open_clip is unpinned and absent
    # here) -- ViT-H-14 config only
    return F.gelu(x)


def _act(name):
    return gelu_erf if name == "erf" else quick_gelu


def mha(x, in_w, in_b, out_w, out_b, heads, attn_mask=None):
    """nn.MultiheadAttention(x, x, x, need_weights=False) with batch_first=False.

    Same op sequence as torch's multi_head_attention_forward slow path:
    packed in-projection, view into (bsz*heads), SDPA, permute back, out-proj.
    x: [L, B, E] (LND, clip/model.py:224).
    """
    L, B, E = x.shape
    hd = E // heads
    proj = F.linear(x, in_w, in_b)
    proj = proj.unflatten(-1, (3, E)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
    q, k, v = proj[0], proj[1], proj[2]
    q = q.view(L, B * heads, hd).transpose(0, 1)
    k = k.view(L, B * heads, hd).transpose(0, 1)
    v = v.view(L, B * heads, hd).transpose(0, 1)
    if attn_mask is not None:
        attn_mask = attn_mask.unsqueeze(0).unsqueeze(0)     # [1,1,L,S]
    q = q.view(B, heads, L, hd)
    k = k.view(B, heads, L, hd)
    v = v.view(B, heads, L, hd)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask, 0.0, False)
    o = o.permute(2, 0, 1, 3).contiguous().view(B * L, E)
    o = F.linear(o, out_w, out_b)
    return o.view(L, B, o.size(1))


def residual_block(x, sd, p, heads, attn_mask=None, act="quick"):
    # clip/model.py:183-186 (act: clip/model.py:160-162 QuickGELU, or "erf")
    h = layer_norm(x, _t(sd, p + "ln_1.weight"), _t(sd, p + "ln_1.bias"))
    x = x + mha(h, _t(sd, p + "attn.in_proj_weight"), _t(sd, p + "attn.in_proj_bias"),
                _t(sd, p + "attn.out_proj.weight"), _t(sd, p + "attn.out_proj.bias"),
                heads, attn_mask)
    h = layer_norm(x, _t(sd, p + "ln_2.weight"), _t(sd, p + "ln_2.bias"))
    h = F.linear(h, _t(sd, p + "mlp.c_fc.weight"), _t(sd, p + "mlp.c_fc.bias"))
    h = _act(act)(h)
    h = F.linear(h, _t(sd, p + "mlp.c_proj.weight"), _t(sd, p + "mlp.c_proj.bias"))
    return x + h


@torch.no_grad()
def encode_image(sd, cfg, images):
    """Reference CLIP.encode_image (clip/model.py:335-336 -> 216-235). Returns [B, Wv]."""
    x = images if isinstance(images, torch.Tensor) else torch.from_numpy(images)
    x = x.float()
    P = cfg.vision_patch_size
    x = F.conv2d(x, _t(sd, "visual.conv1.weight"), None, stride=P)
    x = x.reshape(x.shape[0], x.shape[1], -1).permute(0, 2, 1)
    cls = _t(sd, "visual.class_embedding")
    x = torch.cat([cls.to(x.dtype) + torch.zeros(x.shape[0], 1, x.shape[-1], dtype=x.dtype), x], dim=1)
    x = x + _t(sd, "visual.positional_embedding").to(x.dtype)
    x = layer_norm(x, _t(sd, "visual.ln_pre.weight"), _t(sd, "visual.ln_pre.bias"))
    x = x.permute(1, 0, 2)
    for i in range(cfg.vision_layers):
        x = residual_block(x, sd, f"visual.transformer.resblocks.{i}.", cfg.vision_heads,
                           act=cfg.act)
    x = x.permute(1, 0, 2)
    return layer_norm(x[:, 0, :], _t(sd, "visual.ln_post.weight"), _t(sd, "visual.ln_post.bias"))


def causal_mask(n):
    # clip/model.py:323-329
    m = torch.empty(n, n)
    m.fill_(float("-inf"))
    m.triu_(1)
    return m


@torch.no_grad()
def encode_text(sd, cfg, tokens):
    """Reference CLIP.encode_text (clip/model.py:338-353): (x_before [P,Wt], x [P,E])."""
    text = tokens if isinstance(tokens, torch.Tensor) else torch.from_numpy(tokens)
    text = text.long()
    x = F.embedding(text, _t(sd, "token_embedding.weight")).float()
    x = x + _t(sd, "positional_embedding").float()
    x = x.permute(1, 0, 2)
    mask = causal_mask(cfg.context_length)
    for i in range(cfg.transformer_layers):
        x = residual_block(x, sd, f"transformer.resblocks.{i}.", cfg.transformer_heads, mask,
                           act=cfg.act)
    x = x.permute(1, 0, 2)
    x = layer_norm(x, _t(sd, "ln_final.weight"), _t(sd, "ln_final.bias"))
    x_before = x[torch.arange(x.shape[0]), text.argmax(dim=-1)]
    return x_before, x_before @ _t(sd, "text_projection")


@torch.no_grad()
def class_text_weights(sd, cfg, tokens_per_class):
    """clip_classifier (utils.py:31-57): per class normalise, mean over templates,
    renormalise; stack -> [E, C]. tokens_per_class: list of [T,77] token arrays."""
    ws = []
    for toks in tokens_per_class:
        _, emb = encode_text(sd, cfg, toks)
        emb = emb / emb.norm(dim=-1, keepdim=True)
        e = emb.mean(dim=0)
        ws.append(e / e.norm())
    return torch.stack(ws, dim=1)


@torch.no_grad()
def zero_shot_logits(x_before, vit_proj, text_weights, scale=100.0):
    """methods/ProLIP.py:38-41 + 288-291: (x @ proj) -> F.normalize -> scale * f @ W."""
    f = x_before @ (vit_proj if isinstance(vit_proj, torch.Tensor) else torch.from_numpy(vit_proj))
    f = F.normalize(f, dim=-1)
    return scale * f @ text_weights


def normalize(x):
    # aihab_utils/feature_cache.py:126-127 (F.normalize, eps 1e-12)
    return F.normalize(x, dim=-1)


def topk(logits, k):
    # methods/utils.py:16-21 (topk largest, sorted)
    return logits.topk(k, 1, True, True)[1]


def margins(logits):
    """top1 - top2 logit gap per row: the parity budget for bit-exact top-1."""
    v = logits.topk(2, 1, True, True)[0]
    return v[:, 0] - v[:, 1]


def gflop_per_image(cfg):
    W, L, N, P = cfg.vision_width, cfg.vision_layers, cfg.n_tokens, cfg.vision_patch_size
    return (2 * (N - 1) * 3 * P * P * W + L * (24 * N * W * W + 4 * N * N * W)) / 1e9

