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

// fp16-in -> compute-dtype-out LayerNorm for the fp16 residual stream (the
// per-block ln_1 / ln_2 and in-place ln_pre): two rows per wave, a half-wave
// per row, 8 values per lane per 256 columns, so every load and store is 16 B
// (the general kernel moves 8 B per lane for fp16). Sums over the 32 lanes of
// a half-wave: half_sum (common.h; DPP, then v_permlane16_swap for the last step).

// MX = true: MX-fp8 output (the fp8 GEMM's A operand) instead of T; a 32-value
// block is the 4 lanes of a quad here (8 values per lane), scale by lane 0 of it.
// A workgroup takes kLnRows consecutive rows (each wave kLnRows / 4, two at a
// time): gamma / beta are staged in LDS once per workgroup instead of being
// re-loaded (4 x 16 B per lane per 256 columns) for every row pair.
constexpr int kLnRows = 32;

template <int NI, typename T, bool MX, int ROWS = kLnRows>
__global__ __launch_bounds__(256) void layernorm_h2_kernel(const _Float16* in,  // may alias out
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           T* out, int R, int D,
                                                           uint8_t* __restrict__ oq,
                                                           uint8_t* __restrict__ os) {
  __shared__ float4 gb[2][NI * 64];
  for (int t = threadIdx.x; t < NI * 64; t += 256) {
    gb[0][t] = ((const float4*)gamma)[t];
    gb[1][t] = ((const float4*)beta)[t];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int wave = threadIdx.x >> 6;
  constexpr int PAIRS = ROWS / 8;      // row pairs per wave
  for (int it = 0; it < PAIRS; ++it) {
    const int p2 = ((blockIdx.x * 4 + wave) * PAIRS + it) * 2;   // first row of the pair
    if (p2 >= R) break;                                          // wave-uniform
    const int r = p2 + (lane >> 5);
    const bool valid = r < R;
    const _Float16* src = in + (size_t)(valid ? r : R - 1) * D + hl * 8;
    float v[NI][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const i16x8 h = *(const i16x8*)(src + i * 256);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = from_bits<_Float16>(h[e]);
      s += ((v[i][0] + v[i][1]) + (v[i][2] + v[i][3])) + ((v[i][4] + v[i][5]) + (v[i][6] + v[i][7]));
    }
    const float mean = half_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[i][e] -= mean;
        q += v[i][e] * v[i][e];
      }
    const float rstd = rsqrtf(half_sum(q) / (float)D + 1e-5f);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int c = i * 256 + hl * 8;
      const float4 g0 = gb[0][c / 4], g1 = gb[0][c / 4 + 1];
      const float4 b0 = gb[1][c / 4], b1 = gb[1][c / 4 + 1];
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      if constexpr (MX) {
        float y[8];
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          y[e] = v[i][e] * rstd * g[e] + b[e];
          a = fmaxf(a, fabsf(y[e]));
        }
        a = fmaxf(a, dppf<0xB1>(a));   // quad_perm [1,0,3,2]
        a = fmaxf(a, dppf<0x4E>(a));   // quad_perm [2,3,0,1]: the quad's 32 values
        const int ex = mx_exponent(a);
        const unsigned lo = mx_pack4(make_float4(y[0], y[1], y[2], y[3]), ex);
        const unsigned hi = mx_pack4(make_float4(y[4], y[5], y[6], y[7]), ex);
        if (valid) {
          *(uint2*)(oq + (size_t)r * D + c) = make_uint2(lo, hi);
          if ((hl & 3) == 0) os[mx_scale_index(r, c >> 5, D / 128)] = (uint8_t)(ex + 127);
        }
      } else {
        i16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = to_bits<T>(v[i][e] * rstd * g[e] + b[e]);
        if (valid) *(i16x8*)(out + (size_t)r * D + c) = o;
      }
    }
  }
}

// Statistics only (folded LayerNorm, epilogue.h EpiStoreLN): the same rows per
// wave, loads and reductions as layernorm_h2_kernel, so {mean, rstd} are the
// values that kernel normalises with; one 8-byte store per row.
// rscale (nullable): the folded weight's 1/S (ln_fold), a power of two, so
// {mean, rstd / S} is exact and the GEMM epilogue needs no extra multiply.
template <int NI>
__global__ __launch_bounds__(256) void ln_stats_kernel(const _Float16* __restrict__ in,
                                                       float2* __restrict__ stats, int R, int D,
                                                       const float* __restrict__ rscale) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int r = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if ((blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 >= R) return;
  const bool valid = r < R;
  const _Float16* src = in + (size_t)(valid ? r : R - 1) * D + hl * 8;
  float v[NI][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const i16x8 h = *(const i16x8*)(src + i * 256);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = from_bits<_Float16>(h[e]);
    s += ((v[i][0] + v[i][1]) + (v[i][2] + v[i][3])) + ((v[i][4] + v[i][5]) + (v[i][6] + v[i][7]));
  }
  const float mean = half_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[i][e] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(half_sum(q) / (float)D + 1e-5f);
  if (valid && hl == 0) stats[r] = make_float2(mean, rscale ? rstd * *rscale : rstd);
}

// max |W[j,k] * gamma[k]| over the matrix, as the bits of a non-negative float
// (ordered like unsigned ints) in *amax, which the caller zeroes.
template <typename T>
__global__ __launch_bounds__(256) void fold_amax_kernel(const T* __restrict__ W,
                                                        const float* __restrict__ gamma,
                                                        unsigned* __restrict__ amax, int N, int K) {
  float m = 0.f;
  const size_t n = (size_t)N * K;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    m = fmaxf(m, fabsf((float)W[i] * gamma[i % K]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(amax, __float_as_uint(m));
}

// S = 2^(15 - E) for amax = f * 2^E, f in [0.5, 1): the largest folded weight
// lands in [2^14, 2^15], well inside fp16's range, so small gamma never pushes
// W * gamma into the fp16 subnormals (the reference applies gamma in fp32,
// clip/model.py:154-157). Exact power of two: dividing it back out is exact.
MICLIP_DEV float fold_scale(unsigned amax_bits) {
  const float a = __uint_as_float(amax_bits);
  if (!(a > 0.f) || !(a < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(a, &e);
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  return ldexpf(1.f, 15 - e);
}

// One workgroup per output row j: Wf[j,:] = W[j,:] * gamma * S, colsum[j] = sum Wf[j,:],
// c[j] = bias[j] + beta . W[j,:]; per-thread double partials, fixed-order LDS tree.
// Block 0 also stores 1/S (the ln_stats rscale of this weight) when inv_scale is set.
template <typename T>
__global__ __launch_bounds__(256) void ln_fold_kernel(const T* __restrict__ W,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      const float* __restrict__ bias,
                                                      T* __restrict__ Wf, float* __restrict__ colsum,
                                                      float* __restrict__ c, int K,
                                                      const unsigned* __restrict__ amax,
                                                      float* __restrict__ inv_scale) {
  __shared__ double red[2][256];
  const int j = blockIdx.x, t = threadIdx.x;
  const float S = amax ? fold_scale(*amax) : 1.f;
  if (inv_scale && j == 0 && t == 0) *inv_scale = 1.f / S;
  double ps = 0.0, pc = 0.0;
  for (int k = t; k < K; k += 256) {
    const float w = (float)W[(size_t)j * K + k];
    const T wf = (T)((w * gamma[k]) * S);
    Wf[(size_t)j * K + k] = wf;
    ps += (double)(float)wf;
    pc += (double)beta[k] * (double)w;
  }
  red[0][t] = ps;
  red[1][t] = pc;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) {
      red[0][t] += red[0][t + h];
      red[1][t] += red[1][t + h];
    }
    __syncthreads();
  }
  if (t == 0) {
    colsum[j] = (float)red[0][0];
    c[j] = (float)(red[1][0] + (bias ? (double)bias[j] : 0.0));
  }
}

// Rows per workgroup: 32 (gamma / beta staged once for 32 rows) while that still
// gives every CU a few workgroups; 8 for smaller launches, where 32-row workgroups
// leave ~6 waves per CU and the row loads' latency shows (ViT-B/32 bs=256: 12 800
// rows = 400 workgroups of 32), and 8 for the MX-fp8 output at any size (its
// quantisation math leaves 5 waves per SIMD at 32 rows; C5's 131 584 x 1280 launch:
// 0.098-0.099 vs 0.111 ms, 8 / 16 / 32 rows, 3 interleaved rounds,
// profiles/r05/ln_mx_rows/). The arithmetic per row is the same.
template <typename T, bool MX = false>
hipError_t ln_h2_dispatch(const _Float16* in, const float* g, const float* b, void* out, int R,
                          int D, hipStream_t s, void* oq = nullptr, void* os = nullptr) {
  const bool small = MX || (R + kLnRows - 1) / kLnRows < 1024;
  const dim3 grid(small ? (R + 7) / 8 : (R + kLnRows - 1) / kLnRows), block(256);
#define MICLIP_LNH_CASE(V)                                                                      \
  case V:                                                                                       \
    if (small)                                                                                  \
      hipLaunchKernelGGL((layernorm_h2_kernel<V, T, MX, 8>), grid, block, 0, s, in, g, b,       \
                         (T*)out, R, D, (uint8_t*)oq, (uint8_t*)os);                            \
    else                                                                                        \
      hipLaunchKernelGGL((layernorm_h2_kernel<V, T, MX>), grid, block, 0, s, in, g, b, (T*)out, \
                         R, D, (uint8_t*)oq, (uint8_t*)os);                                     \
    break;
  switch (D / 256) {
    MICLIP_LNH_CASE(1)
    MICLIP_LNH_CASE(2)
    MICLIP_LNH_CASE(3)
    MICLIP_LNH_CASE(4)
    MICLIP_LNH_CASE(5)
    MICLIP_LNH_CASE(6)
    default:
      return hipErrorInvalidValue;
  }
#undef MICLIP_LNH_CASE
  return hipGetLastError();
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

hipError_t ln_stats(const void* in, float* stats, int R, int D, hipStream_t s,
                    const float* rscale) {
  if (R < 1 || D % 256 || D > 1536 || !in || !stats) return hipErrorInvalidValue;
  const dim3 grid((R + 7) / 8), block(256);
#define MICLIP_LNS_CASE(V)                                                              \
  case V:                                                                               \
    hipLaunchKernelGGL((ln_stats_kernel<V>), grid, block, 0, s, (const _Float16*)in,    \
                       (float2*)stats, R, D, rscale);                                   \
    break;
  switch (D / 256) {
    MICLIP_LNS_CASE(1)
    MICLIP_LNS_CASE(2)
    MICLIP_LNS_CASE(3)
    MICLIP_LNS_CASE(4)
    MICLIP_LNS_CASE(5)
    MICLIP_LNS_CASE(6)
    default:
      return hipErrorInvalidValue;
  }
#undef MICLIP_LNS_CASE
  return hipGetLastError();
}

hipError_t ln_fold(int dtype, const void* W, const float* gamma, const float* beta,
                   const float* bias, void* Wf, float* colsum, float* c, int N, int K,
                   hipStream_t s, float* inv_scale) {
  if (N < 1 || K < 1 || !W || !gamma || !beta || !Wf || !colsum || !c) return hipErrorInvalidValue;
  // inv_scale is a device float[2]: [0] receives 1/S, [1] is the amax scratch word
  unsigned* amax = inv_scale ? (unsigned*)(inv_scale + 1) : nullptr;
  if (amax) {
    hipError_t e = hipMemsetAsync(amax, 0, sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    const size_t want = ((size_t)N * K + 4095) / 4096;   // >= 16 elements per thread
    const int blocks = (int)(want < 1024 ? want : 1024);
    if (dtype == kF16)
      hipLaunchKernelGGL((fold_amax_kernel<_Float16>), dim3(blocks), dim3(256), 0, s,
                         (const _Float16*)W, gamma, amax, N, K);
    else
      hipLaunchKernelGGL((fold_amax_kernel<__bf16>), dim3(blocks), dim3(256), 0, s,
                         (const __bf16*)W, gamma, amax, N, K);
  }
  if (dtype == kF16)
    hipLaunchKernelGGL((ln_fold_kernel<_Float16>), dim3(N), dim3(256), 0, s, (const _Float16*)W,
                       gamma, beta, bias, (_Float16*)Wf, colsum, c, K, amax, inv_scale);
  else
    hipLaunchKernelGGL((ln_fold_kernel<__bf16>), dim3(N), dim3(256), 0, s, (const __bf16*)W,
                       gamma, beta, bias, (__bf16*)Wf, colsum, c, K, amax, inv_scale);
  return hipGetLastError();
}

hipError_t layernorm(int dtype, const void* in, const int32_t* rows, int in_stride_rows,
                     const float* gamma, const float* beta, float* out_f32, void* out_t, int R,
                     int D, int normalize, hipStream_t s, int in16, void* out_q, void* out_s) {
  if (R < 1 || D % 256 || D > 1536 || (!out_f32 && !out_t && !out_q)) return hipErrorInvalidValue;
  if (out_q && !out_s) return hipErrorInvalidValue;
  uint8_t *oq = (uint8_t*)out_q, *os = (uint8_t*)out_s;
  if (in16 && dtype == kBF16) {  // fp16 residual stream under bf16 compute: bf16 out
    if (out_q) return hipErrorInvalidValue;   // MX output: the fp16 models only
    if (out_t && !out_f32 && !rows && in_stride_rows == 1 && !normalize)
      return ln_h2_dispatch<__bf16>((const _Float16*)in, gamma, beta, out_t, R, D, s);
    return ln_dispatch<__bf16>((const _Float16*)in, rows, in_stride_rows, gamma, beta, out_f32,
                               out_t, R, D, normalize, s, oq, os);
  }
  if (in16) {  // fp16 residual stream, fp16 compute (dtype = the out_t type)
    if (dtype != kF16) return hipErrorInvalidValue;
    if (out_t && !out_f32 && !out_q && !rows && in_stride_rows == 1 && !normalize)
      return ln_h2_dispatch<_Float16>((const _Float16*)in, gamma, beta, out_t, R, D, s);
    if (out_q && !out_f32 && !out_t && !rows && in_stride_rows == 1 && !normalize)
      return ln_h2_dispatch<_Float16, true>((const _Float16*)in, gamma, beta, nullptr, R, D, s,
                                            out_q, out_s);
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
