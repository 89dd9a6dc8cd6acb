"""CPU: the MX-fp8 oracle (oracle/mx_oracle.py) on known answers. Parity
unpinned with respect to the reference (no fp8 path there); these pin the
format rules the GPU tests (tests/test_gpu_mx.py) are checked against."""
import numpy as np

from oracle import mx_oracle


def test_scale_index_is_a_bijection_per_plane():
    R, K = 600, 1280
    r, kb = np.meshgrid(np.arange(R), np.arange(K // 32), indexing="ij")
    idx = mx_oracle.scale_index(r, kb, K // 128).ravel()
    assert len(np.unique(idx)) == idx.size
    assert idx.max() < mx_oracle.scale_plane_bytes(R, K)
    # a lane's 8 A scales (rows wr*128 + qi*64 + i*16 + fr, same k-block) are contiguous
    rows = np.array([qi * 64 + i * 16 + 5 for qi in range(2) for i in range(4)])
    assert np.array_equal(np.diff(mx_oracle.scale_index(rows, 2, 10)), np.ones(7))


def test_known_answers():
    x = np.zeros((1, 64), dtype=np.float32)
    x[0, :4] = [448.0, 1.0, -0.5, 0.0]          # amax 448 -> E = 0, exact elements
    x[0, 32:36] = [449.0, 1.0, 1.0625, 3.0]     # amax 449 -> E = 1: 224.5 -> 224, 0.5, 0.53125 -> 0.5 (RNE)
    q, E = mx_oracle.quantize(x)
    assert E.tolist() == [[0, 1]]
    d = mx_oracle.dequantize(q, E)
    assert d[0, :4].tolist() == [448.0, 1.0, -0.5, 0.0]
    assert d[0, 32:36].tolist() == [448.0, 1.0, 1.0, 3.0]
    assert mx_oracle.mx_exponent(np.float32(0.0)) == -127
    assert mx_oracle.mx_exponent(np.float32(896.0)) == 1
    assert mx_oracle.mx_exponent(np.float32(896.5)) == 2


def test_round_trip_bound_and_plane_io():
    g = np.random.default_rng(0)
    x = (g.standard_normal((37, 256)) * np.exp2(g.integers(-8, 8, (37, 8))).repeat(32, 1)).astype(np.float32)
    q, E = mx_oracle.quantize(x)
    d = mx_oracle.dequantize(q, E)
    step = np.ldexp(1.0, E).repeat(32, axis=1)
    assert np.all(np.abs(d - x) <= np.maximum(np.abs(x) * 2.0 ** -4, step * 2.0 ** -10))
    assert np.all(np.abs(x).reshape(37, 8, 32).max(-1) <= 448 * np.ldexp(1.0, E))
    assert np.array_equal(mx_oracle.read_plane(mx_oracle.write_plane(E, 256), 37, 256), E)
