"""Text-side zero-shot head builder: `clip_classifier` (utils.py:31-57).

Per class: format the templates, tokenize, encode_text on the HIP path,
normalise each prompt embedding, mean over templates, renormalise; stack to
text_weights [E, C]. Returns (first-template tokens [C, 77], x_before stacked
[T, C, Wt], text_weights [E, C]) like the reference.

`compute_text_weights_from_tokens` is the open_clip path's reduction over one
flattened [C*T, 77] prompt batch (methods/PEFT_openclip.py:17-47,
aihab_utils/model_init.py:83-101): one encode_text call, normalise, mean over
templates, renormalise, transpose to [E, C].
"""
import torch
import torch.nn.functional as F


def _embed_text(clip_model, tokens):
    """(x_before, x) whatever the model's surface: the miclip open_clip surface
    returns one tensor from encode_text, its `_encode_text` still has both."""
    if getattr(clip_model, "surface", "openai") == "open_clip":
        return clip_model._encode_text(tokens)
    return clip_model.encode_text(tokens)


@torch.no_grad()
def clip_classifier(classnames, template, clip_model, tokenize=None):
    if tokenize is None:
        from . import tokenize
    device = next(clip_model.parameters()).device
    weights, before, first = [], [], []
    for classname in classnames:
        classname = classname.replace("_", " ")
        texts = tokenize([t.format(classname) for t in template]).to(device)
        x_before, emb = _embed_text(clip_model, texts)
        emb /= emb.norm(dim=-1, keepdim=True)
        e = emb.mean(dim=0)
        e /= e.norm()
        weights.append(e)
        before.append(x_before.squeeze(dim=1))
        first.append(texts[0])
    return torch.stack(first, dim=0), torch.stack(before, dim=1), torch.stack(weights, dim=1)


@torch.no_grad()
def text_weights_from_tokens(clip_model, tokens_per_class):
    """Same reduction from pre-tokenised prompts: list of [T, 77] LongTensors."""
    device = next(clip_model.parameters()).device
    ws = []
    for toks in tokens_per_class:
        _, emb = _embed_text(clip_model, toks.to(device))
        emb = emb / emb.norm(dim=-1, keepdim=True)
        e = emb.mean(dim=0)
        ws.append(e / e.norm())
    return torch.stack(ws, dim=1)


@torch.no_grad()
def compute_text_weights_from_tokens(model, prompt_tokens, num_classes: int, num_templates: int):
    """text_weights [E, C] from [num_classes * num_templates, 77] prompt tokens
    (methods/PEFT_openclip.py:17-47): one batched encode_text on the HIP path."""
    expected = int(num_classes) * int(num_templates)
    if int(prompt_tokens.shape[0]) != expected:
        raise ValueError(
            f"Prompt token count mismatch: got {int(prompt_tokens.shape[0])}, "
            f"expected {expected} (= num_classes {num_classes} * num_templates {num_templates}).")
    device = next(model.parameters()).device
    _, feats = _embed_text(model, prompt_tokens.to(device))
    feats = F.normalize(feats, dim=-1)
    feats = feats.view(num_classes, num_templates, feats.shape[-1]).mean(dim=1)
    return F.normalize(feats, dim=-1).t().contiguous()
