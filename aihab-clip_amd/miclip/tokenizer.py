"""Byte-level BPE tokenizer and `tokenize` (host-side string work).

Restates the algorithm of the reference `SimpleTokenizer`
(clip/simple_tokenizer.py:62-132: byte->unicode table, word-final "</w>"
merges over the 49152 ranked merges of bpe_simple_vocab_16e6, special tokens
<|startoftext|>=49406 / <|endoftext|>=49407) and of `tokenize`
(clip/clip.py:192-228: SOT + ids + EOT, zero-padded to 77, RuntimeError when too
long unless truncate). Text cleaning uses html.unescape + whitespace collapse;
`ftfy.fix_text` is applied when ftfy is importable (it is not in this image;
for plain-ASCII prompts it is the identity).

The BPE merge table is data, not code: it is read from MICLIP_BPE_PATH, or from
a copy of `bpe_simple_vocab_16e6.txt.gz` next to this file. No vocabulary file
ships with the repo; the parity tests use committed token-id fixtures.
"""
import gzip
import html
import os
from functools import lru_cache

import regex as re
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))


def default_bpe():
    for p in (os.environ.get("MICLIP_BPE_PATH"), os.path.join(_HERE, "bpe_simple_vocab_16e6.txt.gz")):
        if p and os.path.isfile(p):
            return p
    raise FileNotFoundError("BPE vocabulary not found: set MICLIP_BPE_PATH to "
                            "bpe_simple_vocab_16e6.txt.gz (the CLIP merge table)")


@lru_cache()
def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def _clean(text):
    try:
        import ftfy
        text = ftfy.fix_text(text)
    except ImportError:
        pass
    text = html.unescape(html.unescape(text)).strip()
    return re.sub(r"\s+", " ", text).strip()


class SimpleTokenizer:
    def __init__(self, bpe_path: str = None):
        self.byte_encoder = bytes_to_unicode()
        with gzip.open(bpe_path or default_bpe()) as f:
            merges = f.read().decode("utf-8").split("\n")
        merges = [tuple(m.split()) for m in merges[1:49152 - 256 - 2 + 1]]
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab]
        vocab += ["".join(m) for m in merges]
        vocab += ["<|startoftext|>", "<|endoftext|>"]
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {"<|startoftext|>": "<|startoftext|>", "<|endoftext|>": "<|endoftext|>"}
        self.pat = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|"""
                              r"""[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""", re.IGNORECASE)

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        while len(word) > 1:
            pairs = {(word[i], word[i + 1]) for i in range(len(word) - 1)}
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            a, b = best
            out, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(word[i])
                    i += 1
            word = tuple(out)
        res = " ".join(word)
        self.cache[token] = res
        return res

    def encode(self, text):
        ids = []
        for tok in re.findall(self.pat, _clean(text).lower()):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(tok).split(" "))
        return ids


_tok = None


def tokenize(texts, context_length: int = 77, truncate: bool = False) -> torch.LongTensor:
    """clip.tokenize counterpart (clip/clip.py:192-228)."""
    global _tok
    if _tok is None:
        _tok = SimpleTokenizer()
    if isinstance(texts, str):
        texts = [texts]
    sot, eot = _tok.encoder["<|startoftext|>"], _tok.encoder["<|endoftext|>"]
    result = torch.zeros(len(texts), context_length, dtype=torch.long)
    for i, t in enumerate(texts):
        ids = [sot] + _tok.encode(t) + [eot]
        if len(ids) > context_length:
            if truncate:
                ids = ids[:context_length]
                ids[-1] = eot
            else:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
        result[i, :len(ids)] = torch.tensor(ids)
    return result
