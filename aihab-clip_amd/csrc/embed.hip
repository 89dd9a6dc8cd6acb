// Embedding, gather and head kernels around the transformer stacks.
//
//   im2col       conv1 patchify as a GEMM operand (clip/model.py:204, 217-219)
//   class_token  class-embedding row + pos[0] (clip/model.py:220-221)
//   token_embed  token_embedding(text) + positional_embedding and the EOT index
//                text.argmax(-1) (clip/model.py:339-341, 350)
//   rowvec_matmul  x_before @ text_projection (clip/model.py:351), fp32
//   zero_shot    x @ visual.proj -> F.normalize -> scale * f @ text_weights -> topk
//                (methods/ProLIP.py:38-41, 288-293; methods/utils.py:16-21), fp32
// All of these are small next to the transformer blocks; they are written for
// coalesced access and one launch each, not for MFMA.
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

__global__ __launch_bounds__(256) void rowvec_matmul_kernel(const float* __restrict__ in,
                                                            const float* __restrict__ Wm,
                                                            float* __restrict__ out, int D,
                                                            int E) {
  extern __shared__ float xs[];
  const int r = blockIdx.y;
  for (int d = threadIdx.x; d < D; d += blockDim.x) xs[d] = in[(size_t)r * D + d];
  __syncthreads();
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  float acc = 0.f;
  for (int d = 0; d < D; ++d) acc = fmaf(xs[d], Wm[(size_t)d * E + e], acc);
  out[(size_t)r * E + e] = acc;
}

// out[b, e] = sum_d x[b, d] * W[d, e] (fp32), ROWS rows x 64 columns per
// workgroup: each W element read (coalesced, 256 B per wave) feeds ROWS FMAs;
// the 4 waves split d into quarters and the partials are summed in a fixed
// order (deterministic). Grid: (ceil(B/ROWS), ceil(E/64)) -- enough workgroups
// to spread visual.proj over the chip (B=256, E=768: 384 workgroups).
template <int ROWS>
__global__ __launch_bounds__(256) void rows_matmul_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ W,
                                                          float* __restrict__ out, int B,
                                                          int Din, int E) {
  extern __shared__ float sm[];
  float* xs = sm;                   // [ROWS][Din]
  float* red = xs + ROWS * Din;     // [4][ROWS][64]
  const int b0 = blockIdx.x * ROWS, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nr = B - b0 < ROWS ? B - b0 : ROWS;
  const int col = blockIdx.y * 64 + lane;
  for (int i = tid; i < ROWS * Din; i += 256) {
    const int r = i / Din;
    xs[i] = r < nr ? x[(size_t)(b0 + r) * Din + (i - r * Din)] : 0.f;
  }
  __syncthreads();
  float acc[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
  const int q = (Din + 3) / 4, d0 = w * q, d1 = d0 + q < Din ? d0 + q : Din;
  if (col < E) {
    int d = d0;
    for (; d + 8 <= d1; d += 8) {
      float wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) wv[u] = W[(size_t)(d + u) * E + col];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = fmaf(xs[r * Din + d + u], wv[u], acc[r]);
    }
    for (; d < d1; ++d) {
      const float wv = W[(size_t)d * E + col];
#pragma unroll
      for (int r = 0; r < ROWS; ++r) acc[r] = fmaf(xs[r * Din + d], wv, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r) red[(w * ROWS + r) * 64 + lane] = acc[r];
  __syncthreads();
  for (int i = tid; i < nr * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    if (blockIdx.y * 64 + c < E)
      out[(size_t)(b0 + r) * E + blockIdx.y * 64 + c] =
          (red[(0 * ROWS + r) * 64 + c] + red[(1 * ROWS + r) * 64 + c]) +
          (red[(2 * ROWS + r) * 64 + c] + red[(3 * ROWS + r) * 64 + c]);
  }
}

// ROWS images per workgroup: L2-normalise, logits = scale * f @ tw, top-k. With
// proj != null the projection runs here too (only used when the caller gives
// no scratch for rows_matmul_kernel).
template <int ROWS>
__global__ __launch_bounds__(256) void zero_shot_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ proj,
                                                        const float* __restrict__ tw,
                                                        float* __restrict__ logits,
                                                        int32_t* __restrict__ topk, int B,
                                                        int Din, int E, int C, float scale,
                                                        int k) {
  extern __shared__ float sm[];
  float* xs = sm;                 // [ROWS][Din]
  float* fs = xs + ROWS * Din;    // [ROWS][E]
  float* ls = fs + ROWS * E;      // [ROWS][C]
  float* red = ls + ROWS * C;     // [ROWS][4] partial norms, then [ROWS] inverse norms
  const int b0 = blockIdx.x * ROWS, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nr = B - b0 < ROWS ? B - b0 : ROWS;
  for (int i = tid; i < ROWS * Din; i += 256) {
    const int r = i / Din;
    xs[i] = r < nr ? x[(size_t)(b0 + r) * Din + (i - r * Din)] : 0.f;
  }
  __syncthreads();
  float n2[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) n2[r] = 0.f;
  for (int e = tid; e < E; e += 256) {
    float acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = proj ? 0.f : xs[r * Din + e];
    if (proj) {
      for (int d = 0; d < Din; ++d) {
        const float wv = proj[(size_t)d * E + e];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = fmaf(xs[r * Din + d], wv, acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      fs[r * E + e] = acc[r];
      n2[r] += acc[r] * acc[r];
    }
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const float v = wave_sum(n2[r]);
    if (lane == 0) red[r * 4 + w] = v;
  }
  __syncthreads();
  if (tid < ROWS) {
    const float t = red[tid * 4] + red[tid * 4 + 1] + red[tid * 4 + 2] + red[tid * 4 + 3];
    red[ROWS * 4 + tid] = 1.0f / fmaxf(sqrtf(t), 1e-12f);   // F.normalize eps
  }
  __syncthreads();
  for (int i = tid; i < nr * C; i += 256) {
    const int r = i / C, c = i - r * C;
    const float inv = red[ROWS * 4 + r];
    float acc = 0.f;
    int e = 0;
    for (; e + 8 <= E; e += 8) {
      float tv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) tv[u] = tw[(size_t)(e + u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fmaf(fs[r * E + e + u] * inv, tv[u], acc);
    }
    for (; e < E; ++e) acc = fmaf(fs[r * E + e] * inv, tw[(size_t)e * C + c], acc);
    ls[r * C + c] = scale * acc;
    logits[(size_t)(b0 + r) * C + c] = scale * acc;
  }
  __syncthreads();
  if (topk && tid < nr) {
    // selection of the k largest, ties -> lower index first (sorted, largest first)
    float* l = ls + tid * C;
    for (int j = 0; j < k; ++j) {
      int bi = -1;
      float bv = -INFINITY;
      for (int c = 0; c < C; ++c) {
        const float v = l[c];
        if (bi < 0 || v > bv) { bv = v; bi = c; }
      }
      topk[(size_t)(b0 + tid) * k + j] = bi;
      l[bi] = -INFINITY;
    }
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

template <typename T>
static hipError_t im2col_t(int in_dtype, const void* img, T* patches, int B, int R, int P, int Kp,
                           hipStream_t s) {
  const int np = (R / P) * (R / P);
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
                  int Kp, hipStream_t s) {
  if (B < 1 || P < 1 || R % P || Kp < 3 * P * P) return hipErrorInvalidValue;
  if (dtype == kF16) return im2col_t(in_dtype, img, (_Float16*)patches, B, R, P, Kp, s);
  return im2col_t(in_dtype, img, (__bf16*)patches, B, R, P, Kp, s);
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
  if (R < 1 || D < 1 || E < 1) return hipErrorInvalidValue;
  if ((size_t)(8 * D + 4 * 8 * 64) * sizeof(float) <= 64 * 1024) {
    hipLaunchKernelGGL(rows_matmul_kernel<8>, dim3((R + 7) / 8, (E + 63) / 64), dim3(256),
                       (size_t)(8 * D + 4 * 8 * 64) * sizeof(float), s, in, Wm, out, R, D, E);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(rowvec_matmul_kernel, dim3((E + 255) / 256, R), dim3(256),
                     D * sizeof(float), s, in, Wm, out, D, E);
  return hipGetLastError();
}

hipError_t zero_shot(const float* x, const float* proj, const float* tw, float* logits,
                     int32_t* topk, int B, int Din, int E, int C, float scale, int k,
                     hipStream_t s, float* scratch) {
  if (B < 1 || C < 1 || E < 1 || k < 0 || k > C || (!proj && Din != E)) return hipErrorInvalidValue;
  if (proj && scratch && (size_t)8 * Din * 4 + 4 * 8 * 64 * 4 <= 64 * 1024) {
    // projection spread over the chip, then the head on the projected rows
    hipLaunchKernelGGL(rows_matmul_kernel<8>, dim3((B + 7) / 8, (E + 63) / 64), dim3(256),
                       (size_t)(8 * Din + 4 * 8 * 64) * sizeof(float), s, x, proj, scratch, B,
                       Din, E);
    x = scratch;
    proj = nullptr;
    Din = E;
  }
  const size_t per_row = (size_t)(Din + E + C + 5) * sizeof(float);
  if (8 * per_row <= 64 * 1024) {
    hipLaunchKernelGGL(zero_shot_kernel<8>, dim3((B + 7) / 8), dim3(256), 8 * per_row, s, x, proj,
                       tw, logits, topk, B, Din, E, C, scale, k);
  } else if (per_row <= 64 * 1024) {
    hipLaunchKernelGGL(zero_shot_kernel<1>, dim3(B), dim3(256), per_row, s, x, proj, tw, logits,
                       topk, B, Din, E, C, scale, k);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace miclip
