"""Text-side zero-shot head builder: `clip_classifier` (utils.py:31-57).

Per class: format the templates, tokenize, encode_text on the HIP path,
normalise each prompt embedding, mean over templates, renormalise; stack to
text_weights [E, C]. Returns (first-template tokens [C, 77], x_before stacked
[T, C, Wt], text_weights [E, C]) like the reference.
"""
import torch


@torch.no_grad()
def clip_classifier(classnames, template, clip_model, tokenize=None):
    if tokenize is None:
        from . import tokenize
    device = next(clip_model.parameters()).device
    weights, before, first = [], [], []
    for classname in classnames:
        classname = classname.replace("_", " ")
        texts = tokenize([t.format(classname) for t in template]).to(device)
        x_before, emb = clip_model.encode_text(texts)
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
        _, emb = clip_model.encode_text(toks.to(device))
        emb = emb / emb.norm(dim=-1, keepdim=True)
        e = emb.mean(dim=0)
        ws.append(e / e.norm())
    return torch.stack(ws, dim=1)
