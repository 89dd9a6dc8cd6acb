// LayerNorm with fp32 statistics (reference LayerNorm, clip/model.py:151-157:
// upcast to fp32, nn.LayerNorm eps=1e-5, affine) and the optional row L2
// normalisation of the feature cache (F.normalize, eps 1e-12;
// aihab_utils/feature_cache.py:126-127).
//
// HBM-bound: one wave per row, the row held in registers (D/64 floats per
// lane, float4 loads), two-pass mean/variance from registers (no re-read),
// wave-shuffle reductions, vectorised 8/16-byte stores. Row gathers (CLS rows
// for ln_post, EOT rows for ln_final) go through an index array so the
// gathered rows are never materialised.
#include "common.h"
#include "kernels.h"
#include "mx.h"

namespace miclip {

namespace {

// 4 consecutive input elements as fp32 (TI = float, or _Float16 for the fp16
// residual stream: 8-byte loads)
template <typename TI>
MICLIP_DEV float4 load4(const TI* p, size_t i4) {
  if constexpr (std::is_same_v<TI, float>) {
    return ((const float4*)p)[i4];
  } else {
    const i16x4 h = ((const i16x4*)p)[i4];
    return make_float4(from_bits<TI>(h[0]), from_bits<TI>(h[1]), from_bits<TI>(h[2]),
                       from_bits<TI>(h[3]));
  }
}

template <int VPL, typename T, typename TI>  // VPL = float4 vectors per lane (D = 256*VPL)
__global__ __launch_bounds__(256) void layernorm_kernel(const TI* in,  // may alias out_f32 / out_t
                                                        const int32_t* __restrict__ rows,
                                                        int in_stride_rows,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        float* out_f32, T* out_t, int R, int D,
                                                        int normalize, uint8_t* out_q,
                                                        uint8_t* out_s) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const size_t src_row = rows ? (size_t)rows[r] : (size_t)r * in_stride_rows;
  const TI* src = in + src_row * D;
  float4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    v[i] = load4<TI>(src, i * 64 + lane);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    v[i].x -= mean; v[i].y -= mean; v[i].z -= mean; v[i].w -= mean;
    q += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + 1e-5f);
  const float4* g4 = (const float4*)gamma;
  const float4* b4 = (const float4*)beta;
  float n2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float4 g = g4[i * 64 + lane], b = b4[i * 64 + lane];
    v[i].x = v[i].x * rstd * g.x + b.x;
    v[i].y = v[i].y * rstd * g.y + b.y;
    v[i].z = v[i].z * rstd * g.z + b.z;
    v[i].w = v[i].w * rstd * g.w + b.w;
    n2 += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
  }
  if (normalize) {
    const float inv = 1.0f / fmaxf(sqrtf(wave_sum(n2)), 1e-12f);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      v[i].x *= inv; v[i].y *= inv; v[i].z *= inv; v[i].w *= inv;
    }
  }
  if (out_q) {
    // MX-fp8 rows for the fp8 GEMM (gemm_mx.hip): 32-value block = 8 lanes
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      int e;
      const unsigned q = mx_quant4(v[i], e);
      const int k = i * 256 + 4 * lane;
      *(unsigned*)(out_q + (size_t)r * D + k) = q;
      if ((lane & 7) == 0) out_s[mx_scale_index(r, k >> 5, D / 128)] = (uint8_t)(e + 127);
    }
  } else if (out_f32) {
    float4* dst = (float4*)(out_f32 + (size_t)r * D);
#pragma unroll
    for (int i = 0; i < VPL; ++i) dst[i * 64 + lane] = v[i];
  } else {
    i16x4* dst = (i16x4*)(out_t + (size_t)r * D);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      i16x4 o;
      o[0] = to_bits<T>(v[i].x);
      o[1] = to_bits<T>(v[i].y);
      o[2] = to_bits<T>(v[i].z);
      o[3] = to_bits<T>(v[i].w);
      dst[i * 64 + lane] = o;
    }
  }
}

template <typename T, typename TI>
hipError_t ln_dispatch(const TI* in, const int32_t* rows, int stride, const float* g,
                       const float* b, float* of, void* ot, int R, int D, int nz, hipStream_t s,
                       uint8_t* oq, uint8_t* os) {
  const dim3 grid((R + 3) / 4), block(256);
#define MICLIP_LN_CASE(V)                                                                       \
  case V:                                                                                       \
    hipLaunchKernelGGL((layernorm_kernel<V, T, TI>), grid, block, 0, s, in, rows, stride, g, b, \
                       of, (T*)ot, R, D, nz, oq, os);                                           \
    break;
  switch (D / 256) {
    MICLIP_LN_CASE(1)
    MICLIP_LN_CASE(2)
    MICLIP_LN_CASE(3)
    MICLIP_LN_CASE(4)
    MICLIP_LN_CASE(5)
    MICLIP_LN_CASE(6)
    default:
      return hipErrorInvalidValue;
  }
#undef MICLIP_LN_CASE
  return hipGetLastError();
}

}  // namespace

hipError_t layernorm(int dtype, const void* in, const int32_t* rows, int in_stride_rows,
                     const float* gamma, const float* beta, float* out_f32, void* out_t, int R,
                     int D, int normalize, hipStream_t s, int in16, void* out_q, void* out_s) {
  if (R < 1 || D % 256 || D > 1536 || (!out_f32 && !out_t && !out_q)) return hipErrorInvalidValue;
  if (out_q && !out_s) return hipErrorInvalidValue;
  uint8_t *oq = (uint8_t*)out_q, *os = (uint8_t*)out_s;
  if (in16) {  // fp16 residual stream: fp16 compute only
    if (dtype != kF16) return hipErrorInvalidValue;
    return ln_dispatch<_Float16>((const _Float16*)in, rows, in_stride_rows, gamma, beta, out_f32,
                                 out_t, R, D, normalize, s, oq, os);
  }
  if (dtype == kF16)
    return ln_dispatch<_Float16>((const float*)in, rows, in_stride_rows, gamma, beta, out_f32,
                                 out_t, R, D, normalize, s, oq, os);
  return ln_dispatch<__bf16>((const float*)in, rows, in_stride_rows, gamma, beta, out_f32, out_t,
                             R, D, normalize, s, oq, os);
}

}  // namespace miclip
