"""CPU: the C-ABI library loads and exports every symbol include/miclip.h declares.

No compute calls (there is no GPU here); argument validation that happens
before any device access is exercised.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "miclip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(miclip_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from miclip import _lib
    if not os.path.isfile(_lib.LIB_PATH):
        subprocess.run(["make", "-C", ROOT, "-j", "8"], check=True)
    return _lib.load_library()


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("miclip_model_create", "miclip_encode_image", "miclip_encode_text",
              "miclip_zero_shot", "miclip_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    from miclip import _lib
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared_symbols())


def test_nm_shows_c_linkage():
    from miclip import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for s in declared_symbols():
        assert re.search(rf"\bT {s}$", out, flags=re.M), f"{s} not exported with C linkage"


def test_abi_version_and_validation(lib):
    from miclip import _lib
    assert lib.miclip_abi_version() == _lib.ABI_VERSION == 9
    bad = _lib.MiclipConfig(embed_dim=512, image_resolution=224, vision_layers=12, vision_width=700,
                            vision_patch_size=32, context_length=77, vocab_size=49408,
                            transformer_width=512, transformer_heads=8, transformer_layers=12,
                            compute_dtype=0, act=1)
    h = ctypes.c_void_p()
    rc = lib.miclip_model_create(ctypes.byref(bad), 0, ctypes.byref(h))
    assert rc == -1
    assert b"vision_width" in lib.miclip_last_error()
    # open_clip ViT-H/14 heads (80) are accepted, other head widths are not
    bad_dh = _lib.MiclipConfig(embed_dim=1024, image_resolution=224, vision_layers=32,
                               vision_width=1280, vision_patch_size=14, context_length=77,
                               vocab_size=49408, transformer_width=1024, transformer_heads=16,
                               transformer_layers=24, compute_dtype=0, act=2, vision_head_dim=96)
    assert lib.miclip_model_create(ctypes.byref(bad_dh), 0, ctypes.byref(h)) == -1
    assert b"vision_head_dim" in lib.miclip_last_error()
    assert lib.miclip_model_create(None, 0, ctypes.byref(h)) == -1
    assert lib.miclip_op_gemm(0, None, None, None, None, 1, 128, 64, 0, 0, 0, None) == -1
    assert lib.miclip_encode_image_ex(None, None, _lib.MICLIP_F32, 1, None, 0, None) == -1
    assert lib.miclip_clock_probe(None, 8, None) == -1
    lib.miclip_model_destroy(None)           # no-op on NULL
    assert lib.miclip_model_bytes(None) == 0
    assert lib.miclip_model_flags(None) == 0
    assert lib.miclip_model_set_option(None, _lib.MICLIP_OPT_FULL_LAST_BLOCK, 1) == -1
    # unknown option bits are rejected before any device call
    bad_opt = _lib.MiclipConfig(embed_dim=512, image_resolution=224, vision_layers=12,
                                vision_width=768, vision_patch_size=32, context_length=77,
                                vocab_size=49408, transformer_width=512, transformer_heads=8,
                                transformer_layers=12, compute_dtype=0, act=1, options=1 << 9)
    assert lib.miclip_model_create(ctypes.byref(bad_opt), 0, ctypes.byref(h)) == -1
    assert b"options" in lib.miclip_last_error()


def test_product_library_has_no_experimental_kernels():
    """The measured-slower experimental kernels of earlier rounds (ping-pong /
    256x128 / 4-wave GEMMs, streamed attention; numbers in DESIGN.md) were removed
    from the sources; the product libmiclip.so does not contain them."""
    from miclip import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gemm256s_kernel" in data
    for name in (b"gemm_pp_kernel", b"gemm_t2_kernel", b"gemm4w_kernel", b"gemm4s_kernel",
                 b"attention_stream_kernel"):
        assert name not in data, name
