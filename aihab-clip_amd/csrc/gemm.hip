// MFMA GEMM with fused epilogues for the ViT / text ResidualAttentionBlock.
//
// Replaces the torch Linear / packed in-projection / out-projection / conv1
// call sites of the reference (clip/model.py:171-175, 179-181, 204+217 and
// torch.nn.functional multi_head_attention_forward's in/out projections):
//   C[M,N] = A[M,K] . W[N,K]^T, A = activations (token rows), W = nn.Linear weight
//   layout [out, in] -- both operands K-contiguous ("NT"), so both MFMA
//   fragments are 16-byte row reads from LDS.
//
// CDNA4 design (cdna_hip_programming.md §5):
//   * 128x128x64 tile, 256 threads = 4 waves as 2(M) x 2(N), 64x64 per wave,
//     v_mfma_f32_16x16x32_{f16,bf16} with 4x4 fp32 accumulator tiles;
//   * global -> LDS by global_load_lds_dwordx4 (16 B per lane, 1 KiB per wave
//     instruction = 8 rows of 128 B), two LDS stages (64 KiB -> 2 WGs/CU);
//   * LDS image lane-linear, 16-B chunks XOR-swizzled by (row & 7) on the SOURCE
//     address and the same XOR on the ds_read_b128 address (rule 21, T2):
//     conflict-free for the 16x16x32 fragment reads;
//   * all fragments of a K-tile are read before the next tile's DMA is issued,
//     so no ds_read ever waits behind an in-flight LDS-DMA;
//   * bijective XCD-aware block remap so an XCD walks a contiguous range of
//     (A row-panel, W column-panel) tiles (T1).
// Epilogues are fused: bias, bias+QuickGELU (clip/model.py:160-162), bias +
// fp32 residual add (clip/model.py:184-185), and the patch-embed row remap +
// positional-embedding add (clip/model.py:217-221).
#include "common.h"
#include "kernels.h"

namespace miclip {

namespace {

constexpr int BK = 64;

// The activation is a template parameter so that the QKV projection (no
// activation) and the MLP c_fc (QuickGELU) are distinct kernels in a profile.
template <typename T, int ACT>
struct EpiStore {
  T* C;
  const float* bias;
  int ldc;
  MICLIP_DEV void operator()(int r, int c, float v) const {
    if (bias) v += bias[c];
    if (ACT == ACT_QUICKGELU) {
      v = v / (1.0f + __expf(-1.702f * v));
    } else if (ACT == ACT_GELU) {
      v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    }
    C[(size_t)r * ldc + c] = to_t<T>(v);
  }
};

struct EpiResidual {
  float* X;
  const float* bias;
  int ldx;
  MICLIP_DEV void operator()(int r, int c, float v) const {
    float* p = X + (size_t)r * ldx + c;
    *p = *p + (v + bias[c]);
  }
};

struct EpiF32 {
  float* C;
  const float* bias;
  int ldc;
  MICLIP_DEV void operator()(int r, int c, float v) const {
    C[(size_t)r * ldc + c] = bias ? v + bias[c] : v;
  }
};

struct EpiPatch {
  float* X;
  const float* pos;
  int ldx;
  int np;
  MICLIP_DEV void operator()(int r, int c, float v) const {
    const int b = r / np, p = r - b * np;
    const size_t row = (size_t)b * (np + 1) + 1 + p;
    X[row * ldx + c] = v + pos[(size_t)(1 + p) * ldx + c];
  }
};

template <typename T, int BM, int BN, class Epi>
__global__ __launch_bounds__(256) void gemm_nt_kernel(const T* __restrict__ A,
                                                      const T* __restrict__ W, int M, int N,
                                                      int K, Epi epi) {
  constexpr int WN = 2;
  constexpr int TM = BM / 2, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int APW = BM / 8 / 4, BPW = BN / 8 / 4;  // 1 KiB pieces per wave
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int ntn = N / BN, ntm = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, ntm * ntn);
  const int tm = bid / ntn, tn = bid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // DMA sources: lane -> row (lane>>3) of an 8-row piece, physical chunk lane&7,
  // which holds logical chunk (lane&7) ^ (row&7).
  const int prow = lane >> 3, lchunk = (lane & 7) ^ prow;
  const T* a_src[APW];
  const T* b_src[BPW];
#pragma unroll
  for (int p = 0; p < APW; ++p) {
    int row = m0 + (wave * APW + p) * 8 + prow;
    row = row < M ? row : M - 1;
    a_src[p] = A + (size_t)row * K + lchunk * 8;
  }
#pragma unroll
  for (int p = 0; p < BPW; ++p) {
    const int row = n0 + (wave * BPW + p) * 8 + prow;
    b_src[p] = W + (size_t)row * K + lchunk * 8;
  }

  // fragment read offsets (bytes within a stage)
  const int fr = lane & 15, fk = lane >> 4;
  int a_off[FM][2], b_off[FN][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
      a_off[i][s] = (wm * TM + i * 16 + fr) * 128 + (((4 * s + fk) ^ (fr & 7)) << 4);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      b_off[j][s] = A_BYTES + (wn * TN + j * 16 + fr) * 128 + (((4 * s + fk) ^ (fr & 7)) << 4);
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int buf, int k0) {
    char* sa = smem + buf * STAGE;
#pragma unroll
    for (int p = 0; p < APW; ++p) glds16(a_src[p] + k0, sa + (wave * APW + p) * 1024);
#pragma unroll
    for (int p = 0; p < BPW; ++p)
      glds16(b_src[p] + k0, sa + A_BYTES + (wave * BPW + p) * 1024);
  };

  const int nk = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const char* sb = smem + (t & 1) * STAGE;
    i16x8 af[2][FM], bf[2][FN];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < FM; ++i) af[s][i] = *(const i16x8*)(sb + a_off[i][s]);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[s][j] = *(const i16x8*)(sb + b_off[j][s]);
    }
    if (t + 1 < nk) stage((t + 1) & 1, (t + 1) * BK);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = Mfma<T>::m16(af[s][i], bf[s][j], acc[i][j]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * TN + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * TM + i * 16 + fk * 4 + r;
        if (row < M) epi(row, col, acc[i][j][r]);
      }
    }
  }
}

bool gemm_shape_ok(int M, int N, int K) {
  return M >= 1 && N >= 128 && K >= BK && N % 128 == 0 && K % BK == 0;
}

template <typename T, class Epi>
hipError_t launch(const void* A, const void* W, int M, int N, int K, Epi epi, hipStream_t s) {
  if (!gemm_shape_ok(M, N, K)) return hipErrorInvalidValue;
  constexpr int BM = 128, BN = 128;
  const int grid = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, Epi>), dim3(grid), dim3(256), 0, s,
                     (const T*)A, (const T*)W, M, N, K, epi);
  return hipGetLastError();
}

}  // namespace

template <typename T>
hipError_t gemm_store_t(const void* A, const void* W, const float* bias, void* C, int M, int N,
                        int K, int act, hipStream_t s) {
  switch (act) {
    case ACT_NONE:
      return launch<T>(A, W, M, N, K, EpiStore<T, ACT_NONE>{(T*)C, bias, N}, s);
    case ACT_QUICKGELU:
      return launch<T>(A, W, M, N, K, EpiStore<T, ACT_QUICKGELU>{(T*)C, bias, N}, s);
    case ACT_GELU:
      return launch<T>(A, W, M, N, K, EpiStore<T, ACT_GELU>{(T*)C, bias, N}, s);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t gemm_store(int dtype, const void* A, const void* W, const float* bias, void* C, int M,
                      int N, int K, int act, hipStream_t s) {
  if (dtype == kF16) return gemm_store_t<_Float16>(A, W, bias, C, M, N, K, act, s);
  return gemm_store_t<__bf16>(A, W, bias, C, M, N, K, act, s);
}

hipError_t gemm_residual(int dtype, const void* A, const void* W, const float* bias, float* X,
                         int M, int N, int K, hipStream_t s) {
  if (dtype == kF16) return launch<_Float16>(A, W, M, N, K, EpiResidual{X, bias, N}, s);
  return launch<__bf16>(A, W, M, N, K, EpiResidual{X, bias, N}, s);
}

hipError_t gemm_f32(int dtype, const void* A, const void* W, const float* bias, float* C, int M,
                    int N, int K, hipStream_t s) {
  if (dtype == kF16) return launch<_Float16>(A, W, M, N, K, EpiF32{C, bias, N}, s);
  return launch<__bf16>(A, W, M, N, K, EpiF32{C, bias, N}, s);
}

hipError_t gemm_patch(int dtype, const void* A, const void* W, const float* pos, float* X, int M,
                      int N, int K, int np, hipStream_t s) {
  if (np <= 0 || M % np) return hipErrorInvalidValue;
  if (dtype == kF16) return launch<_Float16>(A, W, M, N, K, EpiPatch{X, pos, N, np}, s);
  return launch<__bf16>(A, W, M, N, K, EpiPatch{X, pos, N, np}, s);
}

}  // namespace miclip
