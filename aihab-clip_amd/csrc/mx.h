// MX-fp8 quantisation helpers (OCP MX: e4m3 elements, one E8M0 scale per 32
// consecutive values), shared by the fp8 GEMM epilogue and the LayerNorm MX
// output. A 32-value block is 8 consecutive lanes x 4 values.
#pragma once
#include "common.h"

namespace miclip {

namespace {

// max over the 8 consecutive lanes of a 32-element block (4 elements per lane)
MICLIP_DEV float block8_max(float m) {
  m = fmaxf(m, dppf<0xB1>(m));    // quad_perm [1,0,3,2]
  m = fmaxf(m, dppf<0x4E>(m));    // quad_perm [2,3,0,1]
  m = fmaxf(m, dppf<0x141>(m));   // row_half_mirror: the other quad of the 8
  return m;
}

// E8M0 exponent E = ceil(log2(amax / 448)), clamped to [-127, 126]
MICLIP_DEV int mx_exponent(float amax) {
  const unsigned b = __builtin_bit_cast(unsigned, amax * (1.0f / 448.0f));
  int e = (int)((b >> 23) & 0xff) - 127 + ((b & 0x7fffff) != 0);
  return e < -127 ? -127 : (e > 126 ? 126 : e);
}

// 4 values / 2^E -> 4 packed e4m3 bytes (RNE)
MICLIP_DEV unsigned mx_pack4(float4 v, int e) {
  const float inv = __builtin_bit_cast(float, (unsigned)(127 - e) << 23);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(v.x * inv, v.y * inv, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(v.z * inv, v.w * inv, w, true);
  return (unsigned)w;
}

// Quantise the 4 values this lane holds of a 32-element block spread over 8
// consecutive lanes: returns the packed bytes, `e` the block exponent.
MICLIP_DEV unsigned mx_quant4(float4 v, int& e) {
  const float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
  e = mx_exponent(block8_max(a));
  return mx_pack4(v, e);
}

}  // namespace

}  // namespace miclip
