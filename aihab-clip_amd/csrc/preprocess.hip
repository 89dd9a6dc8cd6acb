// On-device CLIP image preprocessing.
//
// Replaces the reference's per-image CPU transform
//   clip/clip.py:74-81 `_transform` / data/clip_transforms.py:50-55 (test split):
//   Resize(n, BICUBIC) on the shorter side -> CenterCrop(n) -> RGB -> ToTensor
//   -> Normalize(CLIP_MEAN, CLIP_STD)
// whose arithmetic is torchvision's size/anchor rules over Pillow's
// libImaging/Resample.c (8-bit two-pass separable cubic, a = -0.5, fixed point
// with 22 fractional bits). The kernel reproduces it bit for bit on uint8 HWC
// images already in HBM, computing only the crop window:
//   * coefficients are evaluated per workgroup in double with FP contraction
//     off, in Resample.c's operation order (identical doubles to the CPU);
//   * horizontal pass: input rows the band's vertical taps need x crop
//     columns -> uint8 staging rows in LDS (clip8 between passes, as Pillow);
//   * vertical pass from LDS -> clip8 -> float32 x/255, (x-mean)/std
//     (ToTensor + Normalize) written planar [B,3,n,n], or the uint8 crop.
// One workgroup per (image, band of 16 crop rows); the band's vertical span
// is cut into sub-bands that fit the LDS staging area. HBM-bound: each input
// byte of the crop window is read about once (L1/L2 absorb the tap overlap).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "miclip.h"
#include "kernels.h"

namespace miclip {
namespace {

constexpr int kPB = 22;          // Resample.c PRECISION_BITS = 32 - 8 - 2
constexpr int kBand = 16;        // crop rows per workgroup
constexpr int kThreads = 256;

#pragma clang fp contract(off)
__device__ __host__ double cubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Resample.c precompute_coeffs + normalize_coeffs_8bpc for output index xx of
// an in_size -> out_size resize over the whole input; writes ksize fixed-point
// taps (zeros past the count) and returns (xmin, count).
__device__ void coeffs(int in_size, int out_size, int xx, int ksize, int* k, int& xmin_out,
                       int& cnt_out) {
  double filterscale, scale;
  filterscale = scale = (double)in_size / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 2.0 * filterscale;
  const double center = 0.0 + (xx + 0.5) * scale;
  double ww = 0.0;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  for (int x = 0; x < xmax; ++x) ww += cubic((x + xmin - center + 0.5) * ss);
  for (int x = 0; x < ksize; ++x) {
    int v = 0;
    if (x < xmax) {
      double c = cubic((x + xmin - center + 0.5) * ss);   // same double as the sum's term
      if (ww != 0.0) c /= ww;
      const double f = c * (double)(1 << kPB);
      v = c < 0 ? (int)(-0.5 + f) : (int)(0.5 + f);
    }
    k[x] = v;
  }
  xmin_out = xmin;
  cnt_out = xmax;
}

__device__ __forceinline__ int clip8(int v) {
  v >>= kPB;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

struct Geo {
  int nh, nw, top, left;
};

// torchvision: short side -> n, long side -> int(n * long / short); crop anchor
// int(round((size - n) / 2.0)) with Python's half-to-even round.
__device__ __host__ Geo geometry(int h, int w, int n) {
  Geo g;
  if (w <= h) {
    g.nw = n;
    g.nh = (int)((double)((long long)n * h) / w);
  } else {
    g.nh = n;
    g.nw = (int)((double)((long long)n * w) / h);
  }
  g.top = (int)rint((g.nh - n) / 2.0);
  g.left = (int)rint((g.nw - n) / 2.0);
  return g;
}

template <int OUT>  // 0: float32 normalised planar [B,3,n,n]; 1: uint8 crop [B,n,n,3]
__global__ __launch_bounds__(kThreads) void preprocess_kernel(
    const uint8_t* __restrict__ pix, const miclip_image_desc* __restrict__ descs, int n, int KH,
    int KV, int tmp_bytes, void* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* kh = (int*)smem;                      // [n][KH]
  int* khb = kh + n * KH;                    // [n][2] xmin, count
  int* kv = khb + 2 * n;                     // [kBand][KV]
  int* kvb = kv + kBand * KV;                // [kBand][2]
  uint8_t* tmp = (uint8_t*)(kvb + 2 * kBand);

  const int b = blockIdx.x, i0 = blockIdx.y * kBand, tid = threadIdx.x;
  const miclip_image_desc d = descs[b];
  const int H = d.height, W = d.width, C = d.channels;
  const int stride = d.row_stride ? d.row_stride : W * C;
  const uint8_t* img = pix + d.offset;
  const Geo g = geometry(H, W, n);
  const int nrows = n - i0 < kBand ? n - i0 : kBand;

  for (int j = tid; j < n; j += kThreads) {
    int xmin, cnt;
    coeffs(W, g.nw, g.left + j, KH, kh + j * KH, xmin, cnt);
    khb[2 * j] = xmin;
    khb[2 * j + 1] = cnt;
  }
  for (int i = tid; i < nrows; i += kThreads) {
    int ymin, cnt;
    coeffs(H, g.nh, g.top + i0 + i, KV, kv + i * KV, ymin, cnt);
    kvb[2 * i] = ymin;
    kvb[2 * i + 1] = cnt;
  }
  __syncthreads();

  const int rowb = n * C;                    // bytes of one staged row
  const int cap = tmp_bytes / rowb;          // staged rows that fit
  int s0 = 0;
  while (s0 < nrows) {
    // grow the sub-band while its input-row span fits the staging area
    const int ylo = kvb[2 * s0];
    int s1 = s0 + 1;
    while (s1 < nrows && kvb[2 * s1] + kvb[2 * s1 + 1] - ylo <= cap) ++s1;
    const int yhi = kvb[2 * (s1 - 1)] + kvb[2 * (s1 - 1) + 1];
    const int rows = yhi - ylo;

    // horizontal pass: staged[r][j][c] = clip8(half + sum_t in[ylo+r][xmin_j+t][c] * kh[j][t])
    for (int it = tid; it < rows * n; it += kThreads) {
      const int r = it / n, j = it - r * n;
      const int xmin = khb[2 * j], cnt = khb[2 * j + 1];
      const int* k = kh + j * KH;
      const uint8_t* p = img + (size_t)(ylo + r) * stride + (size_t)xmin * C;
      if (C == 3) {
        int a0 = 1 << (kPB - 1), a1 = a0, a2 = a0;
        for (int t = 0; t < cnt; ++t) {
          const int kt = k[t];
          a0 += p[3 * t] * kt;
          a1 += p[3 * t + 1] * kt;
          a2 += p[3 * t + 2] * kt;
        }
        uint8_t* q = tmp + r * rowb + 3 * j;
        q[0] = (uint8_t)clip8(a0);
        q[1] = (uint8_t)clip8(a1);
        q[2] = (uint8_t)clip8(a2);
      } else {
        int a0 = 1 << (kPB - 1);
        for (int t = 0; t < cnt; ++t) a0 += p[t] * k[t];
        tmp[r * rowb + j] = (uint8_t)clip8(a0);
      }
    }
    __syncthreads();

    // vertical pass + ToTensor/Normalize (or the uint8 crop)
    for (int it = tid; it < (s1 - s0) * n; it += kThreads) {
      const int ii = it / n, j = it - ii * n, i = s0 + ii;
      const int ymin = kvb[2 * i] - ylo, cnt = kvb[2 * i + 1];
      const int* k = kv + i * KV;
      int u[3];
      for (int c = 0; c < C; ++c) {
        int a = 1 << (kPB - 1);
        const uint8_t* q = tmp + ymin * rowb + j * C + c;
        for (int t = 0; t < cnt; ++t) a += q[t * rowb] * k[t];
        u[c] = clip8(a);
      }
      if (C == 1) u[1] = u[2] = u[0];   // convert("RGB") of an 'L' image
      const int orow = i0 + i;
      if (OUT == 1) {
        uint8_t* o = (uint8_t*)out + (((size_t)b * n + orow) * n + j) * 3;
        o[0] = (uint8_t)u[0];
        o[1] = (uint8_t)u[1];
        o[2] = (uint8_t)u[2];
      } else {
        // float32(python float) constants, as torch builds the Normalize tensors
        const float mean[3] = {(float)0.48145466, (float)0.4578275, (float)0.40821073};
        const float stdv[3] = {(float)0.26862954, (float)0.26130258, (float)0.27577711};
        float* o = (float*)out + (size_t)b * 3 * n * n + (size_t)orow * n + j;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float x = (float)u[c] / 255.0f;
          o[(size_t)c * n * n] = (x - mean[c]) / stdv[c];
        }
      }
    }
    __syncthreads();
    s0 = s1;
  }
}

int ksize_for(int in_size, int out_size) {
  double fs = (double)in_size / out_size;
  if (fs < 1.0) fs = 1.0;
  return (int)ceil(2.0 * fs) * 2 + 1;
}

}  // namespace

constexpr int kPreTmpBytes = 96 * 1024;

hipError_t preprocess(const uint8_t* pixels, const miclip_image_desc* descs_host,
                      const miclip_image_desc* descs_dev, int B, int n, int out_kind, void* out,
                      hipStream_t s, char* err, int errlen) {
  if (B < 1 || n < 1 || n > 1024 || (out_kind != 0 && out_kind != 1)) {
    snprintf(err, errlen, "preprocess: bad batch %d / resolution %d / output kind %d", B, n,
             out_kind);
    return hipErrorInvalidValue;
  }
  int KH = 1, KV = 1;
  for (int i = 0; i < B; ++i) {
    const miclip_image_desc& d = descs_host[i];
    if (d.height < 1 || d.width < 1 || (d.channels != 1 && d.channels != 3) || d.offset < 0 ||
        (d.row_stride != 0 && d.row_stride < d.width * d.channels)) {
      snprintf(err, errlen, "preprocess: image %d has an invalid descriptor (%dx%dx%d, stride %d)",
               i, d.height, d.width, d.channels, d.row_stride);
      return hipErrorInvalidValue;
    }
    const Geo g = geometry(d.height, d.width, n);
    const int kh = ksize_for(d.width, g.nw), kv = ksize_for(d.height, g.nh);
    KH = kh > KH ? kh : KH;
    KV = kv > KV ? kv : KV;
  }
  // a single crop row's vertical taps must fit the staging area
  if (KH > 64 || KV > 64 || KV > kPreTmpBytes / (n * 3)) {
    snprintf(err, errlen,
             "preprocess: downscale factor too large for resolution %d (taps %d x %d, max 64)", n,
             KH, KV);
    return hipErrorInvalidValue;
  }
  const size_t lds = (size_t)(n * KH + 2 * n + kBand * KV + 2 * kBand) * 4 + kPreTmpBytes;
  if (lds > 160 * 1024) {
    snprintf(err, errlen, "preprocess: LDS need %zu B exceeds 160 KiB", lds);
    return hipErrorInvalidValue;
  }
  const dim3 grid(B, (n + kBand - 1) / kBand);
  if (out_kind == 0) {
    static bool attr0 = hipFuncSetAttribute((const void*)preprocess_kernel<0>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                            160 * 1024) == hipSuccess;
    (void)attr0;
    hipLaunchKernelGGL(preprocess_kernel<0>, grid, dim3(kThreads), lds, s, pixels, descs_dev, n,
                       KH, KV, kPreTmpBytes, out);
  } else {
    static bool attr1 = hipFuncSetAttribute((const void*)preprocess_kernel<1>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                            160 * 1024) == hipSuccess;
    (void)attr1;
    hipLaunchKernelGGL(preprocess_kernel<1>, grid, dim3(kThreads), lds, s, pixels, descs_dev, n,
                       KH, KV, kPreTmpBytes, out);
  }
  return hipGetLastError();
}

}  // namespace miclip
