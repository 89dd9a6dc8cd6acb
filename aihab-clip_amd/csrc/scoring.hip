// Cached-feature consumers on the GPU: the class-centroid
// and multi-prototype outlier scores of tools/outlier_cleaning.py computed
// straight from the embeddings cache.
//
//   * row_norms_kernel       emb.norm(dim=-1)                      (outlier_cleaning.py:234)
//   * class_sums_kernel      sums.index_add_(0, inv, emb)          (:266-267)
//     deterministic: one thread per column walks the class's rows in
//     ascending sample order (CSR built on the host by a stable sort), i.e.
//     the order of the CPU index_add_ -- the sums are bit-identical to it;
//   * centroid_kernel        means = sums / counts -> F.normalize   (:275-276)
//   * proto_score_kernel     sim = x @ protos^T (fp32) fused with the
//     per-sample reductions: best similarity and its prototype among the
//     sample's own class (:626-629, torch.max keeps the first maximum) and
//     best similarity among every other class (:667-673); with inverse norms
//     it is the cosine of score_centroid_distance (:329).
// All fp32 (the reference's dtype). The GEMM-shaped part is tiny next to the
// encoder (N x P x D with P = classes x <= 6 prototypes) and HBM-bound on the
// embeddings read; 64 samples x 64 prototypes per workgroup step, 4 x 4
// outputs per thread from LDS.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kernels.h"

namespace miclip {
namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(64) void row_norms_kernel(const float* __restrict__ x, int D,
                                                       float* __restrict__ norms) {
  const float* row = x + (size_t)blockIdx.x * D;
  float s = 0.f;
  for (int d = threadIdx.x; d < D; d += 64) s = fmaf(row[d], row[d], s);
  s = wsum(s);
  if (threadIdx.x == 0) norms[blockIdx.x] = sqrtf(s);
}

__global__ __launch_bounds__(64) void class_sums_kernel(const float* __restrict__ x,
                                                        const int32_t* __restrict__ order,
                                                        const int32_t* __restrict__ offsets,
                                                        int D, float* __restrict__ sums) {
  const int k = blockIdx.y, col = blockIdx.x * 64 + threadIdx.x;
  if (col >= D) return;
  const int i0 = offsets[k], i1 = offsets[k + 1];
  float acc = 0.f;
  int i = i0;
  for (; i + 8 <= i1; i += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x[(size_t)order[i + u] * D + col];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; i < i1; ++i) acc += x[(size_t)order[i] * D + col];
  sums[(size_t)k * D + col] = acc;
}

// means = sums / count; out = means / max(||means||, eps)  (F.normalize)
__global__ __launch_bounds__(64) void centroid_kernel(const float* __restrict__ sums,
                                                      const int32_t* __restrict__ offsets, int D,
                                                      float eps, float* __restrict__ out) {
  const int k = blockIdx.x;
  const float cnt = (float)(offsets[k + 1] - offsets[k]);
  const float* s = sums + (size_t)k * D;
  float* o = out + (size_t)k * D;
  float n2 = 0.f;
  for (int d = threadIdx.x; d < D; d += 64) {
    const float m = s[d] / cnt;
    o[d] = m;
    n2 = fmaf(m, m, n2);
  }
  const float nrm = fmaxf(sqrtf(wsum(n2)), eps);
  for (int d = threadIdx.x; d < D; d += 64) o[d] = o[d] / nrm;
}

// out = x / max(norm, eps) per row  (outlier_cleaning.py:244)
__global__ __launch_bounds__(256) void div_rows_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ norms, int D,
                                                       float eps, float* __restrict__ out) {
  const float n = fmaxf(norms[blockIdx.x], eps);
  const size_t o = (size_t)blockIdx.x * D;
  for (int d = threadIdx.x; d < D; d += 256) out[o + d] = x[o + d] / n;
}

constexpr int kTS = 64;   // samples per tile
constexpr int kTP = 64;   // prototypes per tile
constexpr int kTK = 16;   // depth per LDS stage

__global__ __launch_bounds__(256) void proto_score_kernel(
    const float* __restrict__ x, const float* __restrict__ protos,
    const int32_t* __restrict__ owner, const int32_t* __restrict__ cls,
    const float* __restrict__ inv_nx, const float* __restrict__ inv_np, int N, int P, int D,
    float* __restrict__ own_best, int32_t* __restrict__ own_arg,
    float* __restrict__ other_best) {
  __shared__ float xs[kTK][kTS + 4];
  __shared__ float ps[kTK][kTP + 4];
  __shared__ float r_own[kTS][16], r_oth[kTS][16];
  __shared__ int r_arg[kTS][16];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int s0 = blockIdx.x * kTS;
  // this thread's 4 samples: rows ty*4 .. +3 of the tile
  int mycls[4];
  float myinv[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int s = s0 + ty * 4 + a;
    mycls[a] = s < N ? cls[s] : -1;
    myinv[a] = (s < N && inv_nx) ? inv_nx[s] : 1.f;
  }
  float best_own[4], best_oth[4];
  int arg_own[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    best_own[a] = -INFINITY;
    best_oth[a] = -INFINITY;
    arg_own[a] = -1;
  }
  const int lr = tid >> 2, lk = (tid & 3) * 4;   // tile loader: row, 4-wide k offset
  for (int p0 = 0; p0 < P; p0 += kTP) {
    float acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
    for (int k0 = 0; k0 < D; k0 += kTK) {
      {
        const int s = s0 + lr, p = p0 + lr;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = k0 + lk + u;
          xs[lk + u][lr] = (s < N && k < D) ? x[(size_t)s * D + k] : 0.f;
          ps[lk + u][lr] = (p < P && k < D) ? protos[(size_t)p * D + k] : 0.f;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kTK; ++k) {
        const float4 xv = *(const float4*)&xs[k][ty * 4];
        const float4 pv = *(const float4*)&ps[k][tx * 4];
        const float xa[4] = {xv.x, xv.y, xv.z, xv.w};
        const float pa[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = fmaf(xa[a], pa[b], acc[a][b]);
      }
      __syncthreads();
    }
    // fold this prototype tile into the running per-sample maxima (ascending
    // prototype order, strict '>' keeps the first maximum like torch.max)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int p = p0 + tx * 4 + b;
      if (p >= P) break;
      const int own = owner[p];
      const float ipn = inv_np ? inv_np[p] : 1.f;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const float v = acc[a][b] * myinv[a] * ipn;
        if (own == mycls[a]) {
          if (v > best_own[a]) { best_own[a] = v; arg_own[a] = p; }
        } else if (v > best_oth[a]) {
          best_oth[a] = v;
        }
      }
    }
  }
  // reduce over the 16 threads (tx) that share each sample; ties -> lowest index
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    r_own[ty * 4 + a][tx] = best_own[a];
    r_oth[ty * 4 + a][tx] = best_oth[a];
    r_arg[ty * 4 + a][tx] = arg_own[a];
  }
  __syncthreads();
  if (tid < kTS) {
    const int s = s0 + tid;
    if (s < N) {
      float bo = -INFINITY, bt = -INFINITY;
      int ba = -1;
      for (int t = 0; t < 16; ++t) {
        const float v = r_own[tid][t];
        const int ar = r_arg[tid][t];
        if (ar >= 0 && (v > bo || (v == bo && (ba < 0 || ar < ba)))) { bo = v; ba = ar; }
        bt = fmaxf(bt, r_oth[tid][t]);
      }
      own_best[s] = bo;
      own_arg[s] = ba;
      other_best[s] = bt;
    }
  }
}

}  // namespace

hipError_t row_norms(const float* x, int N, int D, float* norms, hipStream_t s) {
  if (N < 1 || D < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_norms_kernel, dim3(N), dim3(64), 0, s, x, D, norms);
  return hipGetLastError();
}

hipError_t div_rows(const float* x, const float* norms, int N, int D, float eps, float* out,
                    hipStream_t s) {
  if (N < 1 || D < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(div_rows_kernel, dim3(N), dim3(256), 0, s, x, norms, D, eps, out);
  return hipGetLastError();
}

hipError_t class_centroids(const float* x, const int32_t* order, const int32_t* offsets, int K,
                           int D, float eps, float* sums, float* centroids, hipStream_t s) {
  if (K < 1 || D < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(class_sums_kernel, dim3((D + 63) / 64, K), dim3(64), 0, s, x, order,
                     offsets, D, sums);
  hipLaunchKernelGGL(centroid_kernel, dim3(K), dim3(64), 0, s, sums, offsets, D, eps,
                     centroids);
  return hipGetLastError();
}

hipError_t proto_scores(const float* x, const float* protos, const int32_t* owner,
                        const int32_t* cls, const float* inv_nx, const float* inv_np, int N,
                        int P, int D, float* own_best, int32_t* own_arg, float* other_best,
                        hipStream_t s) {
  if (N < 1 || P < 1 || D < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(proto_score_kernel, dim3((N + kTS - 1) / kTS), dim3(256), 0, s, x, protos,
                     owner, cls, inv_nx, inv_np, N, P, D, own_best, own_arg, other_best);
  return hipGetLastError();
}

}  // namespace miclip
