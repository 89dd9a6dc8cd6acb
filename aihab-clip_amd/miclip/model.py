"""`CLIP` nn.Module whose encoders run on the HIP C ABI (libmiclip.so).

Drop-in for the object the reference's `clip.load` returns (clip/model.py:238-369
built by build_model, clip/model.py:396-433). What callers of the reference
touch, and how it is honoured here:

  * `parameters()` / `named_parameters()` / `state_dict()`: real fp32 torch
    Parameters on the HIP device, named exactly as CLIP.state_dict(), so device
    inference (methods/utils.py:151-153, utils.py:33,
    aihab_utils/feature_cache.py:191) and `state_dict()["visual.proj"]`
    (methods/ProLIP.py:89) work unchanged;
  * `visual.input_resolution`, `visual.output_dim`, `visual.proj`,
    `visual.conv1.weight`, `context_length`, `vocab_size`, `dtype`;
  * `encode_image(image) -> Tensor[B, vision_width]` (pre-projection,
    clip/model.py:228-235) and `encode_text(text) -> (x_before, x)`
    (clip/model.py:338-353). Outputs are fresh, writable fp32 tensors (callers
    divide them in place, utils.py:46-48).

`surface="open_clip"` (the default for open_clip model names such as
"ViT-H-14") gives the same graph open_clip's model surface
instead, the one the PEFT_openclip path calls (methods/PEFT_openclip.py:38-47,
90-92; aihab_utils/feature_cache.py:124-128): `encode_image(image,
normalize=False) -> Tensor[B, embed_dim]` post-projection and
`encode_text(text, normalize=False) -> Tensor[P, embed_dim]` (one tensor), and
`forward` returns open_clip's (image_features, text_features, logit_scale.exp()).

The encoders never run in PyTorch: they call the C ABI, which fails loudly if
the library or the device is missing. The Parameters are the source of truth
for `state_dict`; the handle holds repacked device copies (GEMM weights in the
compute dtype) that are rebuilt whenever the module moves to another device.
"""
import ctypes
import warnings

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from .configs import CLIPConfig

# "mxfp8": QKV / c_fc / c_proj on MX-fp8 operands, fp16 elsewhere
_OUT_FLAGS = {torch.float32: 0, torch.float16: _lib.MICLIP_FLAG_OUT_FP16,
              torch.bfloat16: _lib.MICLIP_FLAG_OUT_BF16}
_DTYPES = {"fp16": (_lib.MICLIP_FP16, torch.float16), "float16": (_lib.MICLIP_FP16, torch.float16),
           "bf16": (_lib.MICLIP_BF16, torch.bfloat16), "bfloat16": (_lib.MICLIP_BF16, torch.bfloat16),
           "mxfp8": (_lib.MICLIP_MXFP8, torch.float16)}


# miclip.load(..., options={...}) / CLIP(..., options=...): the numerics paths of
# include/miclip.h MICLIP_OPT_* (defaults = the benched path). The library reads
# no environment variables; every choice that changes results is named here.
OPTIONS = {
    "resid_f32": (_lib.MICLIP_OPT_RESID_F32, False),        # fp32 residual stream (fp16 compute)
    "ln_fold": (_lib.MICLIP_OPT_NO_LN_FOLD, True),          # ln_1/ln_2 folded into QKV/c_fc
    "mx_out": (_lib.MICLIP_OPT_MX_OUT_FP16, True),          # mxfp8: MX vision out-projection
    "mx_gelu_tanh": (_lib.MICLIP_OPT_MX_GELU_ERF, True),    # mxfp8: tanh-form GELU in MX c_fc
    "cls_last": (_lib.MICLIP_OPT_FULL_LAST_BLOCK, True),    # last vision block on CLS rows
}


def option_bits(options=None):
    """{name: bool} -> MICLIP_OPT_* bits (a bit is set where the value departs
    from the default: the default of every option is 0 bits)."""
    bits = 0
    for k, v in (options or {}).items():
        if k not in OPTIONS:
            raise ValueError(f"unknown miclip option {k!r}; known: {sorted(OPTIONS)}")
        bit, default = OPTIONS[k]
        if bool(v) != default:
            bits |= bit
    return bits


class _Node(nn.Module):
    """Container mirroring one level of the reference module tree."""


class _Handle:
    """Owns one miclip_model* (device-bound)."""

    def __init__(self, cfg: CLIPConfig, compute_dtype: int, device_index: int, options: int = 0):
        self.lib = _lib.load_library()
        c = _lib.MiclipConfig(
            embed_dim=cfg.embed_dim, image_resolution=cfg.image_resolution,
            vision_layers=cfg.vision_layers, vision_width=cfg.vision_width,
            vision_patch_size=cfg.vision_patch_size, context_length=cfg.context_length,
            vocab_size=cfg.vocab_size, transformer_width=cfg.transformer_width,
            transformer_heads=cfg.transformer_heads, transformer_layers=cfg.transformer_layers,
            compute_dtype=compute_dtype,
            act=_lib.MICLIP_ACT_GELU if cfg.act == "erf" else _lib.MICLIP_ACT_QUICKGELU,
            vision_head_dim=cfg.vision_head_width, options=options)
        h = ctypes.c_void_p()
        _lib.check(self.lib.miclip_model_create(ctypes.byref(c), device_index, ctypes.byref(h)),
                   "miclip_model_create")
        self.ptr = h
        self.device_index = device_index

    def load(self, named_arrays):
        keep = []
        arr = (_lib.MiclipTensor * len(named_arrays))()
        for i, (name, a) in enumerate(named_arrays):
            a = np.ascontiguousarray(a, dtype=np.float32)
            keep.append(a)
            arr[i].name = name.encode()
            arr[i].data = a.ctypes.data
            arr[i].numel = a.size
        _lib.check(self.lib.miclip_model_load_weights(self.ptr, arr, len(named_arrays)),
                   "miclip_model_load_weights")

    def load_device(self, named_tensors):
        """Device fp32 tensors on this handle's device: no host round trip."""
        keep = []
        arr = (_lib.MiclipTensor * len(named_tensors))()
        for i, (name, t) in enumerate(named_tensors):
            t = t.detach().to(torch.float32).contiguous()
            if t.device.type != "cuda" or t.device.index != self.device_index:
                raise ValueError(f"{name}: expected a tensor on cuda:{self.device_index}, got {t.device}")
            keep.append(t)
            arr[i].name = name.encode()
            arr[i].data = t.data_ptr()
            arr[i].numel = t.numel()
        torch.cuda.synchronize(self.device_index)      # the tensors' producers are done
        _lib.check(self.lib.miclip_model_load_weights_device(self.ptr, arr, len(named_tensors)),
                   "miclip_model_load_weights_device")

    def close(self):
        if self.ptr:
            self.lib.miclip_model_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


SURFACES = ("openai", "open_clip")


class CLIP(nn.Module):
    def __init__(self, cfg: CLIPConfig, state_dict, device="cuda", compute_dtype="fp16",
                 surface="openai", options=None):
        super().__init__()
        self._options = option_bits(options)
        # runtime settings of the live handle (set_splits / set_gemm_variant /
        # set_profiling; set_cls_last edits _options): re-applied to every new
        # handle, so a device move keeps what the caller chose
        self._splits = None
        self._gemm_variants = {}
        self._profiling = False
        if compute_dtype not in _DTYPES:
            raise ValueError(f"compute_dtype must be one of {sorted(_DTYPES)}")
        if surface not in SURFACES:
            raise ValueError(f"surface must be one of {SURFACES}")
        self.surface = surface
        self.config = cfg
        self.compute_dtype = compute_dtype
        self.context_length = cfg.context_length
        self.vocab_size = cfg.vocab_size
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("miclip encoders run on a HIP device only (got device "
                               f"{dev}); there is no CPU path")
        if not torch.cuda.is_available():
            raise RuntimeError("miclip needs a HIP (ROCm) device; torch.cuda.is_available() is False")
        for name, value in state_dict.items():
            t = value if isinstance(value, torch.Tensor) else torch.from_numpy(np.asarray(value))
            self._register(name, nn.Parameter(t.detach().to(torch.float32).clone(), requires_grad=False))
        self.visual.input_resolution = cfg.image_resolution
        self.visual.output_dim = cfg.embed_dim
        self._handle = None
        self.to(dev)

    # -- module tree -------------------------------------------------------
    def _register(self, dotted, param):
        parts = dotted.split(".")
        mod = self
        for p in parts[:-1]:
            if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                mod.add_module(p, _Node())
            mod = getattr(mod, p)
        mod.register_parameter(parts[-1], param)

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self._sync_handle()
        return out

    def _sync_handle(self):
        p = self.visual.conv1.weight
        if p.device.type != "cuda":
            if self._handle is not None:
                self._handle.close()
            self._handle = None
            return
        idx = p.device.index if p.device.index is not None else torch.cuda.current_device()
        if self._handle is not None and self._handle.device_index == idx:
            return
        if self._handle is not None:
            self._handle.close()
        h = _Handle(self.config, _DTYPES[self.compute_dtype][0], idx, self._options)
        h.load_device(list(self.state_dict().items()))
        self._handle = h
        if self._splits is not None:
            self.set_splits(self._splits)
        for which, variant in self._gemm_variants.items():
            self.set_gemm_variant(which, variant)
        if self._profiling:
            self.set_profiling(True)

    def refresh_weights(self):
        """Re-upload Parameters after they were modified in place (device to device)."""
        if self._handle is not None:
            self._handle.load_device(list(self.state_dict().items()))

    # -- reference surface ---------------------------------------------------
    @property
    def dtype(self):
        # clip/model.py:331-333 returns conv1.weight.dtype, the GPU compute dtype
        return _DTYPES[self.compute_dtype][1]

    @property
    def device(self):
        return self.visual.conv1.weight.device

    @property
    def image_dim(self):
        """Width of encode_image's output: vision_width (OpenAI surface, pre-projection)
        or embed_dim (open_clip surface, post-projection)."""
        return self.config.embed_dim if self.surface == "open_clip" else self.config.vision_width

    def _require(self):
        if self._handle is None:
            raise RuntimeError("model is not on a HIP device; call .cuda() / .to('cuda')")
        return self._handle

    def reserve(self, max_images=0, max_prompts=0):
        h = self._require()
        _lib.check(h.lib.miclip_reserve(h.ptr, int(max_images), int(max_prompts)), "miclip_reserve")

    def set_splits(self, splits=2):
        """Split encode_image batches over 2 HIP streams (default) or not (1)."""
        h = self._require()
        _lib.check(h.lib.miclip_set_splits(h.ptr, int(splits)), "miclip_set_splits")
        self._splits = int(splits)

    def image_splits(self, batch):
        """Parts encode_image splits `batch` images into (miclip_image_splits)."""
        h = self._require()
        n = h.lib.miclip_image_splits(h.ptr, int(batch))
        _lib.check(0 if n > 0 else n, "miclip_image_splits")
        return n

    def numerics(self):
        """The handle's numerics path (miclip_model_flags): every option that changes
        what the kernels compute, as the handle runs it."""
        h = self._require()
        f = h.lib.miclip_model_flags(h.ptr)
        return dict(resid16=bool(f & _lib.MICLIP_MODEL_RESID16),
                    lnfold=bool(f & _lib.MICLIP_MODEL_LNFOLD),          # vision tower
                    lnfold_text=bool(f & _lib.MICLIP_MODEL_LNFOLD_TEXT),
                    mxfp8=bool(f & _lib.MICLIP_MODEL_MXFP8),
                    cls_last=bool(f & _lib.MICLIP_MODEL_CLS_LAST),
                    mx_out=bool(f & _lib.MICLIP_MODEL_MX_OUT),
                    mx_gelu_tanh=bool(f & _lib.MICLIP_MODEL_MX_GELU_TANH))

    def set_gemm_variant(self, which, variant):
        """Diagnostics: kernel of the full-batch GEMM launches (which 0: QKV / c_fc,
        1: out-proj / c_proj, 2: every MX-fp8 GEMM); bit-identical variants only
        (miclip_set_gemm_variant)."""
        h = self._require()
        _lib.check(h.lib.miclip_set_gemm_variant(h.ptr, int(which), int(variant)),
                   "miclip_set_gemm_variant")
        self._gemm_variants[int(which)] = int(variant)

    def set_cls_last(self, on=True):
        """Last vision block on the CLS rows only (default) or over every row."""
        h = self._require()
        _lib.check(h.lib.miclip_model_set_option(h.ptr, _lib.MICLIP_OPT_FULL_LAST_BLOCK,
                                                 int(not on)), "miclip_model_set_option")
        bit = _lib.MICLIP_OPT_FULL_LAST_BLOCK
        self._options = (self._options & ~bit) | (0 if on else bit)

    def set_profiling(self, enable=True):
        h = self._require()
        _lib.check(h.lib.miclip_set_profiling(h.ptr, int(bool(enable))), "miclip_set_profiling")
        self._profiling = bool(enable)

    def profile_read(self, reset=True):
        """{kernel class: dict(launches, ms, flops, bytes)} from the HIP-event profiler."""
        h = self._require()
        arr = (_lib.MiclipKernelStat * 32)()
        n = h.lib.miclip_profile_read(h.ptr, arr, 32, int(bool(reset)))
        if n < 0:
            _lib.check(n, "miclip_profile_read")
        return {arr[i].name.decode(): dict(launches=arr[i].launches, ms=arr[i].ms,
                                           flops=arr[i].flops, bytes=arr[i].bytes)
                for i in range(n) if arr[i].launches}

    # open_clip's training hooks (methods/PEFT_openclip.py:197-273 locks towers and
    # backpropagates through encode_image): outside the inference path built here
    def lock_image_tower(self, *args, **kwargs):
        raise NotImplementedError("miclip is an inference path: open_clip's lock_image_tower / "
                                  "PEFT training (backward through encode_image) is not supported")

    def lock_text_tower(self, *args, **kwargs):
        raise NotImplementedError("miclip is an inference path: open_clip's lock_text_tower / "
                                  "PEFT training is not supported")

    @torch.no_grad()
    def encode_image(self, image, normalize=False, apply_proj=None, out=None, out_dtype=None):
        """Pre-projection image features [B, vision_width] (clip/model.py:335-336, 216-235);
        post-projection [B, embed_dim] on the open_clip surface (open_clip's
        `encode_image(image, normalize=False)`, methods/PEFT_openclip.py:90-92).

        normalize / apply_proj fuse the callers' F.normalize
        (aihab_utils/feature_cache.py:126-127) and `@ visual.proj`
        (methods/ProLIP.py:38-41) into the same launch sequence; apply_proj
        defaults to the surface's contract. out_dtype torch.float32 (default),
        torch.float16 -- the reference GPU path's element type (clip.load on cuda
        keeps the model fp16), so cached f{v}.pth files match its dtype and size --
        or torch.bfloat16: the fp32 result rounded once, in the same launch
        sequence (MICLIP_FLAG_OUT_FP16 / _BF16).
        """
        h = self._require()
        if apply_proj is None:
            apply_proj = self.surface == "open_clip"
        if image.dim() != 4 or image.shape[1] != 3 or image.shape[2] != image.shape[3] \
                or image.shape[2] != self.config.image_resolution:
            raise ValueError(f"expected images [B, 3, {self.config.image_resolution}, "
                             f"{self.config.image_resolution}], got {tuple(image.shape)}")
        # fp16 / bf16 batches are read as they are (miclip_encode_image_ex): the
        # patchify rounds pixels to the compute dtype anyway, so a half batch in
        # the compute dtype gives the fp32 batch's features bit for bit
        in_dt = {torch.float16: _lib.MICLIP_FP16, torch.bfloat16: _lib.MICLIP_BF16}.get(
            image.dtype, _lib.MICLIP_F32)
        img = image.to(device=self.device,
                       dtype=image.dtype if in_dt != _lib.MICLIP_F32 else torch.float32).contiguous()
        B = img.shape[0]
        dim = self.config.embed_dim if apply_proj else self.config.vision_width
        odt = out_dtype if out_dtype is not None else (out.dtype if out is not None else torch.float32)
        oflag = _OUT_FLAGS.get(odt)
        if oflag is None:
            raise ValueError(f"out_dtype must be torch.float32, float16 or bfloat16, got {odt}")
        if out is None:
            out = torch.empty(B, dim, device=self.device, dtype=odt)
        elif out.shape != (B, dim) or out.dtype != odt or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {odt} tensor of shape ({B}, {dim})")
        if B == 0:
            return out
        flags = (_lib.MICLIP_FLAG_NORMALIZE if normalize else 0) | \
                (_lib.MICLIP_FLAG_APPLY_PROJ if apply_proj else 0) | oflag
        with torch.cuda.device(self.device):
            _lib.check(h.lib.miclip_encode_image_ex(h.ptr, img.data_ptr(), in_dt, B, out.data_ptr(),
                                                    flags, _lib.stream_handle(self.device)),
                       "miclip_encode_image_ex")
        return out

    @torch.no_grad()
    def preprocess_images(self, images, uint8=False, out=None):
        """On-device `_transform(R)` (clip/clip.py:74-81) of decoded uint8 images.

        images: a uint8 tensor [B, H, W, C] (any device) or a list of uint8
        HxWxC / HxW arrays or tensors (sizes may differ); C is 3 (RGB) or 1 (L).
        Returns float32 [B, 3, R, R] (ToTensor + Normalize), or with uint8=True
        the resized + center-cropped pixels uint8 [B, R, R, 3]; bit-exact with
        Pillow's bicubic resize + torchvision's crop.
        """
        h = self._require()
        R = self.config.image_resolution
        if isinstance(images, torch.Tensor) and images.dim() == 4:
            if images.dtype != torch.uint8:
                raise ValueError("images must be uint8")
            buf = images.to(self.device).contiguous()
            B, H, W, C = buf.shape
            descs = (_lib.MiclipImageDesc * max(B, 1))(
                *[_lib.MiclipImageDesc(i * H * W * C, H, W, C, 0) for i in range(B)])
        else:
            arrs = []
            for im in images:
                a = im.cpu().numpy() if isinstance(im, torch.Tensor) else np.asarray(im)
                if a.dtype != np.uint8:
                    raise ValueError("images must be uint8")
                if a.ndim == 2:
                    a = a[:, :, None]
                if a.ndim != 3:
                    raise ValueError(f"expected HxWxC images, got shape {a.shape}")
                arrs.append(np.ascontiguousarray(a))
            B = len(arrs)
            offs = np.cumsum([0] + [a.size for a in arrs])
            host = torch.from_numpy(np.concatenate([a.reshape(-1) for a in arrs])) if B else \
                torch.empty(0, dtype=torch.uint8)
            buf = host.pin_memory().to(self.device, non_blocking=True) if B else host
            descs = (_lib.MiclipImageDesc * max(B, 1))(
                *[_lib.MiclipImageDesc(int(offs[i]), a.shape[0], a.shape[1], a.shape[2], 0)
                  for i, a in enumerate(arrs)])
        shape = (B, R, R, 3) if uint8 else (B, 3, R, R)
        dt = torch.uint8 if uint8 else torch.float32
        if out is None:
            out = torch.empty(shape, device=self.device, dtype=dt)
        elif tuple(out.shape) != shape or out.dtype != dt or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {dt} tensor of shape {shape}")
        if B == 0:
            return out
        with torch.cuda.device(self.device):
            _lib.check(h.lib.miclip_preprocess(h.ptr, buf.data_ptr(), descs, B, out.data_ptr(),
                                               _lib.MICLIP_PRE_U8 if uint8 else _lib.MICLIP_PRE_F32,
                                               _lib.stream_handle(self.device)),
                       "miclip_preprocess")
        if buf.is_cuda:
            buf.record_stream(torch.cuda.current_stream(self.device))
        return out

    @torch.no_grad()
    def encode_text(self, text, normalize=False):
        """(x_before_proj [P, transformer_width], x [P, embed_dim]) (clip/model.py:338-353);
        on the open_clip surface one tensor x [P, embed_dim], L2-normalised with
        normalize=True (open_clip's `encode_text(text, normalize=False)`,
        methods/PEFT_openclip.py:38-47)."""
        xb, xp = self._encode_text(text)
        if normalize:
            xp = F.normalize(xp, dim=-1)
        return xp if self.surface == "open_clip" else (xb, xp)

    def _encode_text(self, text):
        h = self._require()
        if text.dim() != 2 or text.shape[1] != self.context_length:
            raise ValueError(f"expected tokens [P, {self.context_length}], got {tuple(text.shape)}")
        if text.device.type == "cpu":
            if text.numel() and (int(text.min()) < 0 or int(text.max()) >= self.vocab_size):
                raise IndexError("index out of range in self (token id outside the vocabulary)")
        tok = text.to(device=self.device, dtype=torch.int64).contiguous()
        P = tok.shape[0]
        xb = torch.empty(P, self.config.transformer_width, device=self.device, dtype=torch.float32)
        xp = torch.empty(P, self.config.embed_dim, device=self.device, dtype=torch.float32)
        if P == 0:
            return xb, xp
        with torch.cuda.device(self.device):
            _lib.check(h.lib.miclip_encode_text(h.ptr, tok.data_ptr(), P, xb.data_ptr(),
                                                xp.data_ptr(), _lib.stream_handle(self.device)),
                       "miclip_encode_text")
        return xb, xp

    @torch.no_grad()
    def zero_shot(self, feats, text_weights, scale=100.0, k=1, apply_proj=True):
        """logits = scale * normalize(feats [@ visual.proj]) @ text_weights and top-k indices.

        methods/ProLIP.py:38-41 + 288-293 (scale 100), methods/utils.py:16-21 (topk).
        """
        h = self._require()
        f = feats.to(device=self.device, dtype=torch.float32).contiguous()
        tw = text_weights.to(device=self.device, dtype=torch.float32).contiguous()
        B, C = f.shape[0], tw.shape[1]
        din = self.config.vision_width if apply_proj else self.config.embed_dim
        if f.dim() != 2 or f.shape[1] != din or tw.shape[0] != self.config.embed_dim:
            raise ValueError(f"feats must be [B, {din}] and text_weights [{self.config.embed_dim}, C]")
        if not 0 <= k <= C:
            raise ValueError(f"k must be in [0, {C}]")
        logits = torch.empty(B, C, device=self.device, dtype=torch.float32)
        top = torch.empty(B, max(k, 1), device=self.device, dtype=torch.int32)
        if B:
            with torch.cuda.device(self.device):
                _lib.check(h.lib.miclip_zero_shot(h.ptr, f.data_ptr(), B, int(bool(apply_proj)),
                                                  tw.data_ptr(), C, float(scale), logits.data_ptr(),
                                                  top.data_ptr() if k else None, int(k),
                                                  _lib.stream_handle(self.device)),
                           "miclip_zero_shot")
        return logits, top[:, :k].long()

    def forward(self, image, text):
        """Upstream CLIP.forward semantics (clip/model.py:355-369) on the joint embedding.

        The vendored forward raises (encode_text returns a tuple);
        this one computes what it was meant to: cosine logits with logit_scale.exp().
        On the open_clip surface: open_clip's (image_features, text_features,
        logit_scale.exp()), both feature sets L2-normalised.
        """
        img = self.encode_image(image, normalize=True, apply_proj=True)
        _, txt = self._encode_text(text)
        if self.surface == "open_clip":
            return img, F.normalize(txt, dim=-1), self.logit_scale.exp()
        txt = txt / txt.norm(dim=-1, keepdim=True)
        logits_per_image = self.logit_scale.exp() * img @ txt.t()
        return logits_per_image, logits_per_image.t()

    def extra_repr(self):
        c = self.config
        return (f"vision=ViT(W={c.vision_width}, L={c.vision_layers}, P={c.vision_patch_size}, "
                f"R={c.image_resolution}), text=(W={c.transformer_width}, L={c.transformer_layers}), "
                f"embed_dim={c.embed_dim}, compute_dtype={self.compute_dtype}, surface={self.surface}")


def build_model(state_dict, device="cuda", compute_dtype="fp16", surface="openai") -> CLIP:
    """Counterpart of reference build_model (clip/model.py:396-433), ViT only."""
    from .configs import config_from_state_dict
    sd = dict(state_dict)
    for key in ("input_resolution", "context_length", "vocab_size"):
        sd.pop(key, None)
    cfg = config_from_state_dict(sd)
    if "logit_scale" not in sd:
        warnings.warn("state_dict has no logit_scale; using log(1/0.07)")
        sd["logit_scale"] = torch.tensor(float(np.log(1 / 0.07)))
    return CLIP(cfg, sd, device=device, compute_dtype=compute_dtype, surface=surface).eval()
