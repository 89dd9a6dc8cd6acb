"""CPU: the MX-fp8 GEMM's inline-asm scale reads keep their address registers.

The K-tile scale reads in gemm_mx.hip are one inline-asm block (ds_read_b64 then
ds_read_b32, then the wait). Without early-clobber outputs hipcc may give the
first read's destination the second read's address register; the second read
then takes its address from a register the first read can overwrite as soon as
its data lands -- a timing-dependent wrong K-tile of W scales (round 3: whole
256-row tiles differing run to run under two streams). This test compiles the
file for gfx950 (device code only, hipcc -S) and checks every such pair in the
emitted code: the b32 read's address register must not be one the b64 read writes.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("make") is None,
                                reason="needs hipcc")

PAIR = re.compile(r"ds_read_b64\s+v\[(\d+):(\d+)\],\s*v(\d+)\s*\n\s*ds_read_b32\s+v(\d+),\s*v(\d+)")


def test_mx_scale_reads_do_not_clobber_their_addresses(tmp_path):
    out = tmp_path / "gemm_mx.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-Wno-unused-function", "-Wno-unused-variable", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "aihab-clip_amd", "csrc", "gemm_mx.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    asm = out.read_text()
    pairs = PAIR.findall(asm)
    assert pairs, "no ds_read_b64/ds_read_b32 scale-read pairs found (asm shape changed?)"
    for lo, hi, _a1, _dst2, a2 in pairs:
        assert not (int(lo) <= int(a2) <= int(hi)), (
            f"ds_read_b32 address v{a2} overwritten by ds_read_b64 v[{lo}:{hi}]")
