// Embedding, gather and head kernels around the transformer stacks.
//
//   im2col       conv1 patchify as a GEMM operand (clip/model.py:204, 217-219)
//   class_token  class-embedding row + pos[0] (clip/model.py:220-221)
//   token_embed  token_embedding(text) + positional_embedding and the EOT index
//                text.argmax(-1) (clip/model.py:339-341, 350)
//   rowvec_matmul  x_before @ text_projection (clip/model.py:351) and
//                x @ visual.proj: fp32 on the f32-input MFMA (head_proj_kernel)
//   zero_shot    x @ visual.proj -> F.normalize -> scale * f @ text_weights -> topk
//                (methods/ProLIP.py:38-41, 288-293; methods/utils.py:16-21), fp32:
//                head_proj_kernel, head_logits_kernel (f32 MFMA, normalise fused),
//                topk_rows_kernel
// All of these are small next to the transformer blocks.
#include "common.h"
#include "kernels.h"

namespace miclip {

namespace {

// I: image element type (fp32, or fp16 / bf16 device-resident input batches)
template <typename T, typename I>
__global__ __launch_bounds__(256) void im2col_kernel(const I* __restrict__ img,
                                                     T* __restrict__ patches, int R, int P,
                                                     int Kp) {
  const int g = R / P, np = g * g;
  const int row = blockIdx.x;  // b*np + py*g + px
  const int b = row / np, pi = row - b * np;
  const int py = pi / g, px = pi - py * g;
  const int PP = P * P, K = 3 * PP;
  const I* src = img + (size_t)b * 3 * R * R + (size_t)(py * P) * R + px * P;
  T* dst = patches + (size_t)row * Kp;
  for (int col = threadIdx.x; col < Kp; col += blockDim.x) {
    float v = 0.f;
    if (col < K) {
      const int c = col / PP, rem = col - c * PP;
      const int ky = rem / P, kx = rem - ky * P;
      v = to_f<I>(src[(size_t)c * R * R + ky * R + kx]);
    }
    dst[col] = to_t<T>(v);
  }
}

// Band form (the default): one workgroup per (image, patch row py). The band's image
// rows py*P .. py*P+P-1 of one channel are ONE contiguous run of P*R elements, so the
// workgroup reads its 3 runs as 4-element vectors (16-B fp32 / 8-B fp16 loads, each
// wave a contiguous 1-KiB / 512-B span; the per-patch kernel above reads one element
// per lane at a P-element stride) and writes each of its g patch rows whole (all three
// channels and the zero pad columns K .. Kp-1). R % 4 == 0 keeps a vector inside one
// image row; its 4 pixels are then PM-aligned runs of one patch row: PM = 4 (P % 4 ==
// 0: one 8-B store), 2 (even P, ViT-L/14: two 4-B stores), 1 (odd P: element stores).
// Same conversion per element as im2col_kernel (bit-identical patches).
template <typename T, typename I, int PM>
__global__ __launch_bounds__(256) void im2col_band_kernel(const I* __restrict__ img,
                                                          T* __restrict__ patches, int R, int P,
                                                          int Kp) {
  const int g = R / P, PP = P * P, K = 3 * PP;
  const int b = blockIdx.x / g, py = blockIdx.x - b * g;
  const int run = P * R, nv = run / 4;
  T* dst0 = patches + ((size_t)b * g + py) * g * Kp;   // patch (b, py, 0)
  const I* src0 = img + (size_t)b * 3 * R * R + (size_t)py * run;
  constexpr int U = 4;   // vectors in flight per lane
  for (int f0 = 0; f0 < 3 * nv; f0 += 256 * U) {
    float v[U][4];
    int fi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      fi[u] = f0 + u * 256 + (int)threadIdx.x;
      const int f = fi[u] < 3 * nv ? fi[u] : 0;
      const int c = f / nv, i = (f - c * nv) * 4;
      const I* p = src0 + (size_t)c * R * R + i;
      if constexpr (sizeof(I) == 4) {
        const float4 x = *(const float4*)p;
        v[u][0] = x.x; v[u][1] = x.y; v[u][2] = x.z; v[u][3] = x.w;
      } else {
        const u32x2 x = *(const u32x2*)p;
        const I* e = (const I*)&x;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[u][k] = to_f<I>(e[k]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (fi[u] >= 3 * nv) continue;
      const int c = fi[u] / nv, i = (fi[u] - c * nv) * 4;
      const int y = i / R, x = i - y * R;
      T o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = to_t<T>(v[u][k]);
      if constexpr (PM == 4) {
        const int px = x / P, kx = x - px * P;
        u32x2 w;
        __builtin_memcpy(&w, o, 8);
        *(u32x2*)(dst0 + (size_t)px * Kp + c * PP + y * P + kx) = w;
      } else if constexpr (PM == 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int xx = x + 2 * h, px = xx / P, kx = xx - px * P;
          unsigned w;
          __builtin_memcpy(&w, o + 2 * h, 4);
          *(unsigned*)(dst0 + (size_t)px * Kp + c * PP + y * P + kx) = w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int xx = x + k, px = xx / P, kx = xx - px * P;
          dst0[(size_t)px * Kp + c * PP + y * P + kx] = o[k];
        }
      }
    }
  }
  const int pad = Kp - K;
  for (int e = threadIdx.x; e < g * pad; e += 256) {
    const int px = e / pad;
    dst0[(size_t)px * Kp + K + (e - px * pad)] = to_t<T>(0.f);
  }
}

// One wave per workgroup: which XCD it runs on, the shader-clock counter
// (s_memtime: free-running at the core clock) and the 100 MHz real-time
// counter. bench.py launches it on the timed stream before and after the timed
// steps; per XCD, delta(s_memtime) / delta(s_memrealtime) x 100 MHz is the
// clock the chip held over the steps. Lane 0 stores (vector stores).
__global__ __launch_bounds__(64) void clock_probe_kernel(unsigned long long* __restrict__ out) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned long long* o = out + 4 * (size_t)blockIdx.x;
    o[0] = xcc & 0xfu;
    o[1] = t;
    o[2] = r;
    o[3] = 0;
  }
}

// R: residual-stream type (float, or _Float16 for the fp16 stream)
template <typename R>
__global__ __launch_bounds__(256) void class_token_kernel(const float* __restrict__ cls,
                                                          const float* __restrict__ pos,
                                                          R* __restrict__ X, int ntok, int D) {
  R* dst = X + (size_t)blockIdx.x * ntok * D;
  for (int d = threadIdx.x; d < D; d += blockDim.x) dst[d] = (R)(cls[d] + pos[d]);
}

template <typename R>
__global__ __launch_bounds__(256) void token_embed_kernel(const int64_t* __restrict__ tokens,
                                                          const float* __restrict__ emb,
                                                          const float* __restrict__ pos,
                                                          R* __restrict__ X, int L, int D,
                                                          int vocab) {
  const int row = blockIdx.x, t = row % L;
  int64_t id = tokens[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // ids are validated on the host
  const float* e = emb + (size_t)id * D;
  const float* p = pos + (size_t)t * D;
  R* dst = X + (size_t)row * D;
  for (int d = threadIdx.x; d < D; d += blockDim.x) dst[d] = (R)(e[d] + p[d]);
}

// one wave per prompt: first index of the maximum token id (torch.argmax)
__global__ __launch_bounds__(64) void eot_kernel(const int64_t* __restrict__ tokens,
                                                 int32_t* __restrict__ eot_rows, int L) {
  const int p = blockIdx.x, lane = threadIdx.x;
  int64_t best = INT64_MIN;
  int bi = 0x7fffffff;
  for (int t = lane; t < L; t += 64) {
    const int64_t v = tokens[(size_t)p * L + t];
    if (v > best) { best = v; bi = t; }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int64_t ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if (lane == 0) eot_rows[p] = p * L + bi;
}

// One wave's share of a 16 x 16 fp32 product on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation): the sum over
// k chunks [c0, c1) of 16 k each of x[row][k] * W[k][col]. Lane (i = lane & 15,
// g = lane >> 4) loads x[row i][16 ch + 4g .. +3] as one float4 (xp = row i + 4g)
// and W[16 ch + 4g + s][col i] for s = 0..3 (wp = W + 4g * ldw + col i); MFMA s
// multiplies the k = 16 ch + 4g + s pairs (the same k permutation on both
// operands), chunks in ascending order. NORM: n2 += the squares of the lane's x
// elements (a row's |x|^2 in the same loop, for the fused normalise).
template <bool NORM>
__device__ __forceinline__ f32x4 mfma_chunks(const float* __restrict__ xp,
                                             const float* __restrict__ wp, size_t ldw, int c0,
                                             int c1, float& n2) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int ch = c0;
  for (; ch + 4 <= c1; ch += 4) {
    float4 a[4];
    float bv[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = *(const float4*)(xp + 16 * (ch + u));
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) bv[u][s2] = wp[(size_t)(16 * (ch + u) + s2) * ldw];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].x, bv[u][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].y, bv[u][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].z, bv[u][2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].w, bv[u][3], acc, 0, 0, 0);
      if (NORM)
        n2 = fmaf(a[u].w, a[u].w, fmaf(a[u].z, a[u].z, fmaf(a[u].y, a[u].y, fmaf(a[u].x, a[u].x, n2))));
    }
  }
  for (; ch < c1; ++ch) {
    const float4 a = *(const float4*)(xp + 16 * ch);
    float bv[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) bv[s2] = wp[(size_t)(16 * ch + s2) * ldw];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bv[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bv[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bv[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bv[3], acc, 0, 0, 0);
    if (NORM) n2 = fmaf(a.w, a.w, fmaf(a.z, a.z, fmaf(a.y, a.y, fmaf(a.x, a.x, n2))));
  }
  return acc;
}

// out[b, e] = sum_d x[b, d] * W[d, e] in fp32 on the f32 MFMA (the projection of
// methods/ProLIP.py:38-41 / clip/model.py:335 and 352). One workgroup = 16 rows x
// 16 columns; wave w takes k chunks [w nk / 4, (w + 1) nk / 4) of the nk = Din / 16,
// and the 4 partial tiles are summed in a fixed order through LDS (deterministic,
// batch-invariant: a row's result does not depend on B). Grid (ceil(B/16),
// ceil(E/16)): 768 workgroups at B = 256, E = 768. Din % 16 == 0.
__global__ __launch_bounds__(256) void head_proj_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ W,
                                                        float* __restrict__ out, int B, int Din,
                                                        int E) {
  __shared__ f32x4 red[3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int b0 = blockIdx.x * 16, c0 = blockIdx.y * 16;
  const int row = b0 + i < B ? b0 + i : B - 1, col = c0 + i < E ? c0 + i : E - 1;
  const int nk = Din / 16;
  float n2 = 0.f;
  const f32x4 acc = mfma_chunks<false>(x + (size_t)row * Din + 4 * g, W + (size_t)(4 * g) * E + col,
                                       E, w * nk / 4, (w + 1) * nk / 4, n2);
  if (w > 0) red[w - 1][lane] = acc;
  __syncthreads();
  if (w > 0) return;
  const f32x4 r1 = red[0][lane], r2 = red[1][lane], r3 = red[2][lane];
  // C layout: lane holds rows 4g .. 4g+3 of column i
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = b0 + 4 * g + j;
    if (r < B && c0 + i < E)
      out[(size_t)r * E + c0 + i] = (acc[j] + r1[j]) + (r2[j] + r3[j]);
  }
}

// The zero-shot logits on the f32 MFMA with the normalise fused (methods/ProLIP.py:
// 288-291, methods/utils.py:16-21): logits[b, c] = scale * (f[b] . tw[:, c]) /
// max(|f[b]|, 1e-12) for f [B, E], tw [E, C]. The tile is head_proj_kernel's (16
// rows x 16 classes, 4 waves over k quarters, fixed-order LDS sum); each lane also
// sums the squares of the f elements it loads for the MFMA, so |f[b]|^2 comes out
// of the same loop (lane groups g in a fixed butterfly, then the 4 waves in a
// fixed order): f is read once, no normalised copy is written. Grid (ceil(B/16),
// ceil(C/16)): 16 x 63 workgroups at B = 256, C = 1000. E % 16 == 0.
__global__ __launch_bounds__(256) void head_logits_kernel(const float* __restrict__ f,
                                                          const float* __restrict__ tw,
                                                          float* __restrict__ logits, int B,
                                                          int E, int C, float scale) {
  __shared__ f32x4 red[3][64];
  __shared__ float nred[4][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int b0 = blockIdx.x * 16, c0 = blockIdx.y * 16;
  const int row = b0 + i < B ? b0 + i : B - 1, col = c0 + i < C ? c0 + i : C - 1;
  const int nk = E / 16;
  float n2 = 0.f;
  const f32x4 acc = mfma_chunks<true>(f + (size_t)row * E + 4 * g, tw + (size_t)(4 * g) * C + col,
                                      C, w * nk / 4, (w + 1) * nk / 4, n2);
  n2 += __shfl_xor(n2, 16);   // (g0 + g1) + (g2 + g3) on every lane of row i
  n2 += __shfl_xor(n2, 32);
  if (g == 0) nred[w][i] = n2;
  if (w > 0) red[w - 1][lane] = acc;
  __syncthreads();
  if (w > 0) return;
  const f32x4 r1 = red[0][lane], r2 = red[1][lane], r3 = red[2][lane];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int rl = 4 * g + j, r = b0 + rl;
    const float nn = (nred[0][rl] + nred[1][rl]) + (nred[2][rl] + nred[3][rl]);
    const float inv = 1.0f / fmaxf(sqrtf(nn), 1e-12f);
    if (r < B && c0 + i < C)
      logits[(size_t)r * C + c0 + i] = scale * (((acc[j] + r1[j]) + (r2[j] + r3[j])) * inv);
  }
}

// The top-k classes of each logits row (largest first, ties -> lower index; the
// order torch.topk(sorted=True) returns for distinct values), one wave per row:
// pick j is the arg-max over the classes strictly after pick j - 1 in (value
// descending, index ascending) order, so no state but the previous pick is kept
// and the row (L2-resident, C floats) is re-read per pick.
__global__ __launch_bounds__(64) void topk_rows_kernel(const float* __restrict__ logits,
                                                       int32_t* __restrict__ topk, int C, int k) {
  const int lane = threadIdx.x;
  const float* lr = logits + (size_t)blockIdx.x * C;
  float pv = INFINITY;
  int pi = -1;
  for (int j = 0; j < k; ++j) {
    float bv = -INFINITY;
    int bi = C;
    for (int c = lane; c < C; c += 64) {
      const float v = lr[c];
      const bool after = v < pv || (v == pv && c > pi);
      if (after && (bi == C || v > bv)) { bv = v; bi = c; }   // ascending c: ties keep the lower
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (oi < C && (bi == C || ov > bv || (ov == bv && oi < bi))) { bv = ov; bi = oi; }
    }
    if (lane == 0) topk[(size_t)blockIdx.x * k + j] = bi;
    pv = bv;
    pi = bi;
  }
}

__global__ __launch_bounds__(64) void row_l2norm_kernel(float* __restrict__ x, int D) {
  float* row = x + (size_t)blockIdx.x * D;
  float n2 = 0.f;
  for (int d = threadIdx.x; d < D; d += 64) n2 += row[d] * row[d];
  const float inv = 1.0f / fmaxf(sqrtf(wave_sum(n2)), 1e-12f);
  for (int d = threadIdx.x; d < D; d += 64) row[d] *= inv;
}

// dst row r = src row r * stride_rows, 16-B chunks (the CLS rows of the residual
// stream for the last vision block, capi.hip run_block_cls)
__global__ void gather_rows_kernel(const char* __restrict__ src, char* __restrict__ dst,
                                   int stride_rows, int row_bytes) {
  const int r = blockIdx.x;
  const char* sp = src + (size_t)r * stride_rows * row_bytes;
  char* dp = dst + (size_t)r * row_bytes;
  for (int c = threadIdx.x * 16; c < row_bytes; c += blockDim.x * 16)
    *(u32x4*)(dp + c) = *(const u32x4*)(sp + c);
}

}  // namespace

// Weight repack at load (convert_weights, clip/model.py:372-393): fp32 rows
// [rows, src_cols] -> compute dtype [rows, cols], zero-padded columns
// (conv1's 3P^2 -> Kp). Round to nearest even, like the reference's .half().
template <typename T>
__global__ __launch_bounds__(256) void cast_pad_kernel(const float* __restrict__ in,
                                                       T* __restrict__ out, int64_t rows,
                                                       int src_cols, int cols) {
  const int64_t n = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    out[i] = (T)(c < src_cols ? in[r * src_cols + c] : 0.f);
  }
}

hipError_t gather_rows(const void* src, void* dst, int R, int stride_rows, int D, int elt_bytes,
                       hipStream_t s) {
  const int row_bytes = D * elt_bytes;
  if (R < 1 || stride_rows < 1 || row_bytes % 16 || (elt_bytes != 2 && elt_bytes != 4))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(R), dim3(256), 0, s, (const char*)src, (char*)dst,
                     stride_rows, row_bytes);
  return hipGetLastError();
}

hipError_t cast_pad(int dtype, const float* in, void* out, int64_t rows, int src_cols, int cols,
                    hipStream_t s) {
  if (!in || !out || rows < 1 || src_cols < 1 || cols < src_cols) return hipErrorInvalidValue;
  const int64_t n = rows * cols;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  if (dtype == kF16)
    hipLaunchKernelGGL((cast_pad_kernel<_Float16>), dim3(grid), dim3(256), 0, s, in,
                       (_Float16*)out, rows, src_cols, cols);
  else
    hipLaunchKernelGGL((cast_pad_kernel<__bf16>), dim3(grid), dim3(256), 0, s, in, (__bf16*)out,
                       rows, src_cols, cols);
  return hipGetLastError();
}

hipError_t row_l2norm(float* x, int R, int D, hipStream_t s) {
  if (R < 1 || D < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_l2norm_kernel, dim3(R), dim3(64), 0, s, x, D);
  return hipGetLastError();
}

template <typename T, typename I>
static void im2col_band(const void* img, T* patches, int B, int R, int P, int Kp, hipStream_t s) {
  const dim3 grid(B * (R / P));
  if (P % 4 == 0)
    hipLaunchKernelGGL((im2col_band_kernel<T, I, 4>), grid, dim3(256), 0, s, (const I*)img, patches,
                       R, P, Kp);
  else if (P % 2 == 0)
    hipLaunchKernelGGL((im2col_band_kernel<T, I, 2>), grid, dim3(256), 0, s, (const I*)img, patches,
                       R, P, Kp);
  else
    hipLaunchKernelGGL((im2col_band_kernel<T, I, 1>), grid, dim3(256), 0, s, (const I*)img, patches,
                       R, P, Kp);
}

// variant 0: the band kernel where it applies (R % 4 == 0, Kp % 4 == 0 and both base
// pointers 16-B aligned: every vector load and store aligned), else the per-patch
// kernel (element accesses, any alignment); 1: the per-patch kernel
template <typename T>
static hipError_t im2col_t(int in_dtype, const void* img, T* patches, int B, int R, int P, int Kp,
                           hipStream_t s, int variant) {
  const int np = (R / P) * (R / P);
  const bool aligned = ((uintptr_t)img & 15) == 0 && ((uintptr_t)patches & 15) == 0;
  if (variant == 0 && aligned && R % 4 == 0 && Kp % 4 == 0 &&
      (in_dtype == kIn32 || in_dtype == kF16 || in_dtype == kBF16)) {
    if (in_dtype == kIn32)
      im2col_band<T, float>(img, patches, B, R, P, Kp, s);
    else if (in_dtype == kF16)
      im2col_band<T, _Float16>(img, patches, B, R, P, Kp, s);
    else
      im2col_band<T, __bf16>(img, patches, B, R, P, Kp, s);
    return hipGetLastError();
  }
  if (in_dtype == kIn32)
    hipLaunchKernelGGL((im2col_kernel<T, float>), dim3(B * np), dim3(256), 0, s,
                       (const float*)img, patches, R, P, Kp);
  else if (in_dtype == kF16)
    hipLaunchKernelGGL((im2col_kernel<T, _Float16>), dim3(B * np), dim3(256), 0, s,
                       (const _Float16*)img, patches, R, P, Kp);
  else if (in_dtype == kBF16)
    hipLaunchKernelGGL((im2col_kernel<T, __bf16>), dim3(B * np), dim3(256), 0, s,
                       (const __bf16*)img, patches, R, P, Kp);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t clock_probe(unsigned long long* out, int n_wg, hipStream_t s) {
  if (!out || n_wg < 1 || n_wg > 4096) return hipErrorInvalidValue;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(n_wg), dim3(64), 0, s, out);
  return hipGetLastError();
}

hipError_t im2col(int dtype, int in_dtype, const void* img, void* patches, int B, int R, int P,
                  int Kp, hipStream_t s, int variant) {
  if (B < 1 || P < 1 || R % P || Kp < 3 * P * P || variant < 0 || variant > 1)
    return hipErrorInvalidValue;
  if (dtype == kF16) return im2col_t(in_dtype, img, (_Float16*)patches, B, R, P, Kp, s, variant);
  return im2col_t(in_dtype, img, (__bf16*)patches, B, R, P, Kp, s, variant);
}

hipError_t class_token(const float* cls, const float* pos, void* X, int B, int ntok, int D,
                       hipStream_t s, int resid16) {
  if (resid16)
    hipLaunchKernelGGL(class_token_kernel<_Float16>, dim3(B), dim3(256), 0, s, cls, pos,
                       (_Float16*)X, ntok, D);
  else
    hipLaunchKernelGGL(class_token_kernel<float>, dim3(B), dim3(256), 0, s, cls, pos, (float*)X,
                       ntok, D);
  return hipGetLastError();
}

hipError_t token_embed(const int64_t* tokens, const float* tok_emb, const float* pos, void* X,
                       int32_t* eot_rows, int P, int L, int D, int vocab, hipStream_t s,
                       int resid16) {
  if (P < 1 || L < 1) return hipErrorInvalidValue;
  if (resid16)
    hipLaunchKernelGGL(token_embed_kernel<_Float16>, dim3(P * L), dim3(256), 0, s, tokens,
                       tok_emb, pos, (_Float16*)X, L, D, vocab);
  else
    hipLaunchKernelGGL(token_embed_kernel<float>, dim3(P * L), dim3(256), 0, s, tokens, tok_emb,
                       pos, (float*)X, L, D, vocab);
  hipLaunchKernelGGL(eot_kernel, dim3(P), dim3(64), 0, s, tokens, eot_rows, L);
  return hipGetLastError();
}

hipError_t rowvec_matmul(const float* in, const float* Wm, float* out, int R, int D, int E,
                         hipStream_t s) {
  if (R < 1 || D < 16 || D % 16 || E < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_proj_kernel, dim3((R + 15) / 16, (E + 15) / 16), dim3(256), 0, s, in,
                     Wm, out, R, D, E);
  return hipGetLastError();
}

hipError_t zero_shot(const float* x, const float* proj, const float* tw, float* logits,
                     int32_t* topk, int B, int Din, int E, int C, float scale, int k,
                     hipStream_t s, float* scratch) {
  if (B < 1 || C < 1 || E < 16 || E % 16 || k < 0 || k > C || (!proj && Din != E) ||
      (proj && !scratch))
    return hipErrorInvalidValue;
  if (proj) {
    // the projection on the f32 MFMA over the whole chip, then the logits
    if (hipError_t e = rowvec_matmul(x, proj, scratch, B, Din, E, s)) return e;
    x = scratch;
  }
  hipLaunchKernelGGL(head_logits_kernel, dim3((B + 15) / 16, (C + 15) / 16), dim3(256), 0, s, x,
                     tw, logits, B, E, C, scale);
  if (topk && k > 0)
    hipLaunchKernelGGL(topk_rows_kernel, dim3(B), dim3(64), 0, s, logits, topk, C, k);
  return hipGetLastError();
}

}  // namespace miclip
