"""ctypes binding of libmiclip.so (the C ABI declared in include/miclip.h).

The product path has no fallback: if the HIP library is missing or cannot be
loaded, every entry point raises. Build it with `make` (or
`python -c "import __graft_entry__ as g; g.build()"`).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MICLIP_LIB", os.path.join(_HERE, "libmiclip.so"))

ABI_VERSION = 9          # include/miclip.h MICLIP_ABI_VERSION
MICLIP_FP16 = 0
MICLIP_BF16 = 1
MICLIP_MXFP8 = 2
MICLIP_F32 = 3
MICLIP_ACT_QUICKGELU = 1
MICLIP_ACT_GELU = 2
MICLIP_FLAG_NORMALIZE = 1
MICLIP_FLAG_APPLY_PROJ = 2
MICLIP_FLAG_OUT_FP16 = 4
MICLIP_FLAG_OUT_BF16 = 8
MICLIP_MODEL_RESID16 = 1
MICLIP_MODEL_LNFOLD = 2
MICLIP_MODEL_MXFP8 = 4
MICLIP_MODEL_CLS_LAST = 8
MICLIP_MODEL_MX_OUT = 16
MICLIP_MODEL_MX_GELU_TANH = 32
MICLIP_MODEL_LNFOLD_TEXT = 64
# miclip_config.options (include/miclip.h MICLIP_OPT_*)
MICLIP_OPT_RESID_F32 = 1
MICLIP_OPT_NO_LN_FOLD = 2
MICLIP_OPT_MX_OUT_FP16 = 4
MICLIP_OPT_MX_GELU_ERF = 8
MICLIP_OPT_FULL_LAST_BLOCK = 16

EXPORTS = (
    "miclip_model_create", "miclip_model_load_weights", "miclip_model_load_weights_device",
    "miclip_reserve",
    "miclip_encode_image", "miclip_encode_image_ex", "miclip_encode_text", "miclip_zero_shot",
    "miclip_clock_probe",
    "miclip_model_destroy", "miclip_last_error", "miclip_abi_version",
    "miclip_model_bytes", "miclip_model_flags", "miclip_model_set_option", "miclip_set_gemm_variant", "miclip_set_profiling", "miclip_profile_read", "miclip_set_splits", "miclip_image_splits",
    "miclip_op_gemm", "miclip_op_gemm_splitk", "miclip_op_ln_stats", "miclip_op_ln_fold", "miclip_op_gemm_ln",
    "miclip_op_layernorm", "miclip_op_attention", "miclip_op_attention_q0", "miclip_op_im2col", "miclip_preprocess",
    "miclip_row_norms", "miclip_class_centroids", "miclip_proto_scores",
    "miclip_mx_scale_bytes", "miclip_op_quant_mx", "miclip_op_gemm_mx", "miclip_op_gemm_mx_v", "miclip_op_layernorm_mx",
)

MICLIP_PRE_F32 = 0
MICLIP_PRE_U8 = 1


class MiclipConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "embed_dim", "image_resolution", "vision_layers", "vision_width", "vision_patch_size",
        "context_length", "vocab_size", "transformer_width", "transformer_heads",
        "transformer_layers", "compute_dtype", "act", "vision_head_dim")] + [
        ("options", ctypes.c_uint32)]


class MiclipTensor(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class MiclipKernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("launches", ctypes.c_int64), ("ms", ctypes.c_double),
                ("flops", ctypes.c_double), ("bytes", ctypes.c_double)]


class MiclipImageDesc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("row_stride", ctypes.c_int32)]


class MiclipError(RuntimeError):
    pass


_lib = None


def load_library(path: str = None):
    """Load (once) and return the ctypes handle; raises MiclipError if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.isfile(p):
        raise MiclipError(f"HIP library not found at {p}; build it with `make` "
                          f"(miclip has no CPU fallback)")
    lib = ctypes.CDLL(p)
    vp, i32, i64, u32, f32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                              ctypes.c_float)
    sig = {
        "miclip_model_create": ([ctypes.POINTER(MiclipConfig), ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "miclip_model_load_weights": ([vp, ctypes.POINTER(MiclipTensor), i32], ctypes.c_int),
        "miclip_model_load_weights_device": ([vp, ctypes.POINTER(MiclipTensor), i32], ctypes.c_int),
        "miclip_reserve": ([vp, i32, i32], ctypes.c_int),
        "miclip_encode_image": ([vp, vp, i32, vp, u32, vp], ctypes.c_int),
        "miclip_encode_image_ex": ([vp, vp, i32, i32, vp, u32, vp], ctypes.c_int),
        "miclip_clock_probe": ([vp, i32, vp], ctypes.c_int),
        "miclip_encode_text": ([vp, vp, i32, vp, vp, vp], ctypes.c_int),
        "miclip_zero_shot": ([vp, vp, i32, i32, vp, i32, f32, vp, vp, i32, vp], ctypes.c_int),
        "miclip_model_destroy": ([vp], None),
        "miclip_last_error": ([], ctypes.c_char_p),
        "miclip_abi_version": ([], ctypes.c_int),
        "miclip_model_bytes": ([vp], i64),
        "miclip_model_flags": ([vp], ctypes.c_int),
        "miclip_model_set_option": ([vp, u32, i32], ctypes.c_int),
        "miclip_set_gemm_variant": ([vp, i32, i32], ctypes.c_int),
        "miclip_set_profiling": ([vp, ctypes.c_int], ctypes.c_int),
        "miclip_set_splits": ([vp, i32], ctypes.c_int),
        "miclip_image_splits": ([vp, i32], ctypes.c_int),
        "miclip_profile_read": ([vp, ctypes.POINTER(MiclipKernelStat), i32, i32], ctypes.c_int),
        "miclip_op_gemm": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], ctypes.c_int),
        "miclip_op_layernorm": ([i32, vp, vp, vp, vp, i32, i32, i32, vp], ctypes.c_int),
        "miclip_op_attention_q0": ([i32, vp, vp, i32, i32, i32, i32, vp], ctypes.c_int),
        "miclip_op_im2col": ([i32, i32, vp, vp, i32, i32, i32, i32, i32, vp], ctypes.c_int),
        "miclip_op_ln_stats": ([vp, vp, i32, i32, vp, vp], ctypes.c_int),
        "miclip_op_ln_fold": ([i32, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp], ctypes.c_int),
        "miclip_op_gemm_splitk": ([i32, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32,
                                   vp, vp], ctypes.c_int),
        "miclip_op_gemm_ln": ([i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
                              ctypes.c_int),
        "miclip_op_attention": ([i32, vp, vp, i32, i32, i32, i32, i32, i32, vp], ctypes.c_int),
        "miclip_mx_scale_bytes": ([i32, i32], i64),
        "miclip_op_quant_mx": ([vp, i32, i32, i32, vp, vp, vp], ctypes.c_int),
        "miclip_op_gemm_mx": ([vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
                              ctypes.c_int),
        "miclip_op_gemm_mx_v": ([vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp],
                                ctypes.c_int),
        "miclip_op_layernorm_mx": ([vp, i32, vp, vp, vp, vp, i32, i32, vp], ctypes.c_int),
        "miclip_preprocess": ([vp, vp, ctypes.POINTER(MiclipImageDesc), i32, vp, i32, vp],
                              ctypes.c_int),
        "miclip_row_norms": ([vp, i32, i32, vp, f32, vp, vp], ctypes.c_int),
        "miclip_class_centroids": ([vp, vp, vp, i32, i32, f32, vp, vp, vp], ctypes.c_int),
        "miclip_proto_scores": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp],
                                ctypes.c_int),
    }
    # an explicitly declared A/B build of an older revision (MICLIP_LIB together with
    # MICLIP_AB_BUILD=1) may predate some op-level entry points: those stay unbound
    # and are named on stderr; any other library -- the product one, or MICLIP_LIB
    # alone -- must export every entry point, or loading fails here
    ab_build = "MICLIP_LIB" in os.environ and os.environ.get("MICLIP_AB_BUILD") == "1"
    unbound = []
    for name, (args, res) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if ab_build and name.startswith("miclip_op_"):
                unbound.append(name)
                continue
            raise
        fn.argtypes = args
        fn.restype = res
    if unbound:
        import sys
        print(f"[miclip] A/B build {os.environ['MICLIP_LIB']}: entry points left unbound: "
              f"{', '.join(unbound)}", file=sys.stderr)
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load_library().miclip_last_error().decode(errors="replace")
        exc = ValueError if rc == -1 else MiclipError
        raise exc(f"{what} failed ({rc}): {msg}")
    return rc


def stream_handle(device=None):
    """Raw hipStream_t of torch's current stream on `device`."""
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
