"""CPU oracle for the MX-fp8 operand format of the MICLIP_MXFP8 path.

TEST INFRASTRUCTURE ONLY (imported by tests/ alone; the product path never
touches it).

Parity unpinned: the reference has no fp8 path at all (the
C5 stretch config asks for fp8 weights on open_clip ViT-H/14 shapes, and
open_clip is absent). What is restated here is the OCP Microscaling (MX) v1.0
format as this build uses it -- e4m3 ("e4m3fn": bias 7, max 448, no infinities)
elements with one E8M0 power-of-two scale per 32 consecutive values of a row --
with this build's scale rule, E = ceil(log2(amax / 448)) (so no element ever
saturates; the spec's floor(log2(amax)) - 8 clamps instead), elements rounded
to nearest-even after the exact power-of-two division (torch's float8_e4m3fn
cast), and the tiled scale-plane layout of aihab-clip_amd/csrc/common.h
`mx_scale_index`.
"""
import numpy as np
import torch


def mx_exponent(amax):
    """E = ceil(log2(amax / 448)) from the fp32 bits of amax * (1/448), clamped [-127, 126]."""
    t = (np.asarray(amax, dtype=np.float32) * np.float32(1.0 / 448.0)).astype(np.float32)
    bits = t.view(np.uint32)
    e = ((bits >> 23) & 0xFF).astype(np.int64) - 127 + ((bits & 0x7FFFFF) != 0)
    return np.clip(e, -127, 126)


def quantize(x):
    """x [R, K] (K % 32 == 0) -> (q uint8 [R, K] e4m3 bytes, E int64 [R, K/32])."""
    x = np.asarray(x, dtype=np.float32)
    R, K = x.shape
    blocks = x.reshape(R, K // 32, 32)
    amax = np.abs(blocks).max(axis=-1)
    E = mx_exponent(amax)
    inv = np.ldexp(np.float32(1.0), -E).astype(np.float32)[..., None]
    y = (blocks * inv).astype(np.float32).reshape(R, K)
    q = torch.from_numpy(y).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    return q, E


def dequantize(q, E):
    q = np.asarray(q, dtype=np.uint8)
    R, K = q.shape
    v = torch.from_numpy(q.copy()).view(torch.float8_e4m3fn).float().numpy()
    return (v.reshape(R, K // 32, 32) * np.ldexp(1.0, E)[..., None]).reshape(R, K).astype(np.float32)


def scale_index(r, kb, KT):
    """common.h mx_scale_index: byte offset of (row r, 32-k block kb) in a tiled plane."""
    r = np.asarray(r, dtype=np.int64)
    kb = np.asarray(kb, dtype=np.int64)
    return ((r >> 8) * KT + (kb >> 2)) * 1024 + (kb & 3) * 256 + (r & 15) * 16 + ((r >> 4) & 15)


def scale_plane_bytes(rows, K):
    return (rows + 255) // 256 * (K // 128) * 1024


def read_plane(plane, R, K):
    """Tiled plane bytes -> E int64 [R, K/32] (valid rows only)."""
    plane = np.asarray(plane, dtype=np.uint8)
    r, kb = np.meshgrid(np.arange(R), np.arange(K // 32), indexing="ij")
    return plane[scale_index(r, kb, K // 128)].astype(np.int64) - 127


def write_plane(E, K):
    R = E.shape[0]
    plane = np.zeros(scale_plane_bytes(R, K), dtype=np.uint8)
    r, kb = np.meshgrid(np.arange(R), np.arange(K // 32), indexing="ij")
    plane[scale_index(r, kb, K // 128)] = (E + 127).astype(np.uint8)
    return plane
