"""Host-side image preprocessing equivalent to the reference `_transform(n_px)`.

clip/clip.py:74-81: Resize(n_px, BICUBIC) on the shorter side -> CenterCrop(n_px)
-> RGB -> ToTensor -> Normalize(CLIP_MEAN, CLIP_STD). torchvision is not in the
image, so this restates it on PIL + numpy. It is host preprocessing (SURVEY §8f
row 1 is the on-device version, out of this round's scope).
"""
import numpy as np
import torch

from .weights import CLIP_MEAN, CLIP_STD


class Transform:
    def __init__(self, n_px: int):
        self.n_px = int(n_px)

    def __call__(self, image):
        from PIL import Image
        if isinstance(image, np.ndarray):
            image = Image.fromarray(image)
        w, h = image.size
        s = self.n_px / min(w, h)
        nw, nh = max(self.n_px, round(w * s)), max(self.n_px, round(h * s))
        image = image.resize((nw, nh), Image.BICUBIC)
        left = int(round((nw - self.n_px) / 2.0))
        top = int(round((nh - self.n_px) / 2.0))
        image = image.crop((left, top, left + self.n_px, top + self.n_px)).convert("RGB")
        a = np.asarray(image, dtype=np.float32) / 255.0                      # ToTensor
        a = (a - np.asarray(CLIP_MEAN, np.float32)) / np.asarray(CLIP_STD, np.float32)
        return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))

    def __repr__(self):
        return (f"Transform(Resize({self.n_px}, bicubic), CenterCrop({self.n_px}), RGB, "
                f"ToTensor, Normalize(mean={CLIP_MEAN}, std={CLIP_STD}))")
