// MX-fp8 GEMM (stretch config C5: fp8 weights for the
// open_clip ViT-H/14 shapes) on gfx950's block-scaled matrix cores.
//
// Operands are OCP MX-fp8: e4m3 elements with one E8M0 (power-of-two) scale per
// 32 consecutive k of a row, i.e. per (row, k-block). The hardware applies the
// scales inside v_mfma_scale_f32_16x16x128_f8f6f4, which runs at twice the
// f16 rate (MI355X_MICROARCH.md, Matrix cores) -- no dequantisation anywhere.
//
// Lane maps (measured: scripts/probe/mx_probe.hip, mx_scale_probe.hip): lane l
// holds row/col l&15; its 8 data VGPRs are the 16-B chunks g and 4+g
// (g = l>>4) of the row's 128-byte K-tile -- the very chunks the f16 kernel's
// two 16x16x32 k-steps read -- and its scale byte is that row's k-block g.
// So one 128-k fp8 K-tile is byte-for-byte the f16 kernel's 64-k K-tile: the
// same LDS-DMA staging, XOR swizzle and fragment reads, one MFMA where the
// f16 kernel issues two, and half as many K-tiles.
//
// Scale planes are tiled for the kernel (mx_scale_index): per (256-row block,
// 128-k tile) one 1-KiB block [k-block 4][row & 15][row >> 4 & 15], so a lane's
// 8 A scales (rows wr*128 + qi*64 + i*16 + fr) are one ds_read_b64 and its 4 W
// scales one ds_read_b32, selected per MFMA by the instruction's byte op_sel.
// The scale blocks ride the A0 half-tile DMA (one global_load_lds_dword per
// wave) into a 2 x 2 KiB LDS ring.
//
// Producers: `quant_mx` (weights at load, any fp32/fp16 rows), the LayerNorm
// MX output (norm.hip) and the EpiMX epilogue below (c_fc + GELU -> MX for
// c_proj). Quantisation rule: E = ceil(log2(amax / 448)) per block, elements
// RNE to e4m3 (v_cvt_pk_fp8_f32) -- no element ever saturates.
#include "common.h"
#include "epilogue.h"
#include "kernels.h"
#include "mx.h"

#include <cstdlib>

namespace miclip {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// c_fc epilogue for the fp8 path: act(acc + bias) quantised to MX-fp8 rows of
// the next GEMM's A operand (data [M, ldc] bytes + tiled scale plane). Called
// by all 64 lanes of a wave with 4 consecutive columns each (the LDS-staged
// epilogue: one row of 256 columns per wave instruction).
template <int ACT>
struct EpiMX {
  uint8_t* C;
  uint8_t* S;
  const float* bias;
  int ldc;
  int kt;  // 128-k tiles per row of the output (= ldc / 128)
  // act(v) on 4 values, the packed forms put4 uses
  MICLIP_DEV static float4 act4(float4 v) {
    if constexpr (ACT == ACT_GELU || ACT == ACT_GELU_TANH || ACT == ACT_QUICKGELU) {
      const f32x2 a = {v.x, v.y}, b = {v.z, v.w};
      const f32x2 lo = ACT == ACT_GELU ? gelu_erf2(a) : ACT == ACT_GELU_TANH ? gelu_tanh2(a) : quick_gelu2(a);
      const f32x2 hi = ACT == ACT_GELU ? gelu_erf2(b) : ACT == ACT_GELU_TANH ? gelu_tanh2(b) : quick_gelu2(b);
      return make_float4(lo[0], lo[1], hi[0], hi[1]);
    } else {
      return v;
    }
  }
  MICLIP_DEV float4 bias4(int col) const { return ld_bias4(bias, col); }
  MICLIP_DEV float4 bias4nb(int col) const { return ld_bias4_nb(bias, col); }
  MICLIP_DEV float bias1(int col) const { return bias ? bias[col] : 0.f; }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4 b) const {
    float4 y;
    if constexpr (ACT == ACT_GELU) {
      const f32x2 lo = gelu_erf2((f32x2){v.x + b.x, v.y + b.y});
      const f32x2 hi = gelu_erf2((f32x2){v.z + b.z, v.w + b.w});
      y = make_float4(lo[0], lo[1], hi[0], hi[1]);
    } else if constexpr (ACT == ACT_GELU_TANH) {
      const f32x2 lo = gelu_tanh2((f32x2){v.x + b.x, v.y + b.y});
      const f32x2 hi = gelu_tanh2((f32x2){v.z + b.z, v.w + b.w});
      y = make_float4(lo[0], lo[1], hi[0], hi[1]);
    } else {
      y = make_float4(act_fn<ACT>(v.x + b.x), act_fn<ACT>(v.y + b.y), act_fn<ACT>(v.z + b.z),
                      act_fn<ACT>(v.w + b.w));
    }
    int e;
    const unsigned q = mx_quant4(y, e);
    *(unsigned*)(C + (size_t)r * ldc + c) = q;
    if ((threadIdx.x & 7) == 0) S[mx_scale_index(r, c >> 5, kt)] = (uint8_t)(e + 127);
  }
};

// 4-byte LDS-DMA of a scale block piece, issued from inline asm: with the
// builtin, hipcc cannot tell the scale ring from the fragment slots and waits
// vmcnt(0) before every scale ds_read (draining the K-tile pipeline). The
// kernel's own counted waits cover it (3 ops per A0 stage). `lds` wave-uniform.
MICLIP_DEV void glds4_hidden(const void* g, const void* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const LDS_AS void*)lds);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(dst)
      : "memory");
}

template <class E> struct IsEpiMX : std::false_type {};
template <int ACT> struct IsEpiMX<EpiMX<ACT>> : std::true_type {};
// fp16 store epilogues (the MX QKV GEMM) also run on transposed accumulators
template <class E> struct IsEpiStoreH : std::false_type {};
template <int ACT> struct IsEpiStoreH<EpiStore<_Float16, ACT>> : std::true_type {};
template <> struct IsEpiStoreH<EpiResidual<_Float16>> : std::true_type {};   // + x at readback

// max over the 4 lanes fr, fr + 16, fr + 32, fr + 48 (the 16-lane rows of a wave):
// one v_permlane16_swap (rows 0<->1, 2<->3) and one v_permlane32_swap
MICLIP_DEV float max_rows4(float m) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  m = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// The scaled MFMAs have no memory side effects, and without a scheduling
// fence hipcc sinks all of a K-tile's MFMAs below the phase barriers (every
// phase's fragments then stay live: 256 VGPRs and spills). sched_barrier(0)
// keeps each phase's MFMAs between its barriers, as in gemm256_kernel.
MICLIP_DEV void lds_barrier_mx() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 256x256x128(fp8) tile, 8 waves 2(M) x 4(N), the staggered 8-phase schedule of
// gemm256_kernel<SCHED 2> (gemm.hip; cdna_hip_programming.md §5 "256^2 8-phase
// template"). vmcnt counts include the scale DMA (3 ops in every A0 stage).
template <class Epi>
__global__ __launch_bounds__(512) void gemm256_mx_kernel(const uint8_t* __restrict__ A,
                                                         const uint8_t* __restrict__ SA,
                                                         const uint8_t* __restrict__ W,
                                                         const uint8_t* __restrict__ SW, int M,
                                                         int N, int K, Epi epi, int gm) {
  constexpr int HALF = 128 * 128;      // bytes of one half-tile slot
  constexpr int EPI_LD = 260;          // fp32 row stride of the epilogue staging
  // MX-fp8 output (EpiMX, c_fc -> c_proj): transposed accumulators (operands
  // swapped, C^T = W . A^T: lane (fk, fr) holds output row fr and 4 consecutive
  // columns 4fk..), so the 32-column MX blocks are quantised in registers
  constexpr bool TR = IsEpiMX<Epi>::value || IsEpiStoreH<Epi>::value;
  constexpr int SCL = 8 * HALF;        // scale ring: 2 x (A 1 KiB + W 1 KiB)
  constexpr int SMEM = 128 * EPI_LD * 4 > SCL + 4096 ? 128 * EPI_LD * 4 : SCL + 4096;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int ntn = N / 256, ntm = (M + 255) / 256, ndp = ntm * ntn;
  const int KT = K / 128, nk = KT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int tm, tn;
  group_tile(xcd_remap(blockIdx.x, ndp), ntm, ntn, gm, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int lchunk = (lane & 7) ^ (lane >> 3);
  const uint8_t* asrc[2][2];
  const uint8_t* bsrc[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int sr = (wave * 2 + pp) * 8 + (lane >> 3);
      int ar = m0 + (sr >> 6) * 128 + h * 64 + (sr & 63);
      ar = ar < M ? ar : M - 1;
      asrc[h][pp] = A + (size_t)ar * K + lchunk * 16;
      const int bc = n0 + (sr >> 5) * 64 + h * 32 + (sr & 31);
      bsrc[h][pp] = W + (size_t)bc * K + lchunk * 16;
    }
  // scale DMA source of this wave: waves 0-3 the A block, 4-7 the W block
  const uint8_t* ssrc = (wave < 4 ? SA + (size_t)tm * KT * 1024 : SW + (size_t)tn * KT * 1024) +
                        (wave & 3) * 256 + lane * 4;
  auto stage = [&](int slot_kind, int tile) {
    const int buf = tile & 1, k0 = tile * 128;
    char* dst = smem + (buf * 4 + slot_kind) * HALF + wave * 2048;
    const uint8_t* const* src = slot_kind < 2 ? asrc[slot_kind] : bsrc[slot_kind - 2];
    glds16(src[0] + k0, dst);
    glds16(src[1] + k0, dst + 1024);
    if (slot_kind == 0)
      glds4_hidden(ssrc + (size_t)tile * 1024,
                   smem + SCL + buf * 2048 + (wave >> 2) * 1024 + (wave & 3) * 256);
  };
  const int fr = lane & 15, fk = lane >> 4;
  const int aoff = (wr * 64 + fr) * 128, boff = (wc * 32 + fr) * 128;
  const int sw0 = ((0 + fk) ^ (fr & 7)) << 4, sw1 = ((4 + fk) ^ (fr & 7)) << 4;
  const int soa = fk * 256 + fr * 16 + wr * 8, sob = 1024 + fk * 256 + fr * 16 + wc * 4;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 8-VGPR fragments: two ds_read_b128 joined into a freshly defined v8i (a
  // partial .lo/.hi update keeps the old tuple live and doubles the registers)
  v8i af[4], bf[2];
  unsigned sa[2], sb = 0;
  auto rd8 = [&](const char* p0, const char* p1) {
    const i32x4 lo = *(const i32x4*)p0, hi = *(const i32x4*)p1;
    return (v8i)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  // phase 2 = (A1, B1) finds B1 still in bf from phase 1: load_b = false there
  auto quadrant = [&](const char* sa_, const char* sb_, bool load_a, bool load_b) {
    if (load_a) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = rd8(sa_ + i * 2048 + sw0, sa_ + i * 2048 + sw1);
    }
    if (load_b) {
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = rd8(sb_ + j * 2048 + sw0, sb_ + j * 2048 + sw1);
    }
  };
  auto mfma_q = [&](int qi, int qj) {
    // op_sel picks the scale byte: A slot qi*4 + i -> dword qi, byte i; W slot
    // qj*2 + j -> byte qj*2 + j, i.e. byte j of sb >> 16*qj. The op_sel values
    // must be immediates, so they depend on the unrolled i / j only.
    const int sca = qi ? (int)sa[1] : (int)sa[0];
    const int scb = qj ? (int)(sb >> 16) : (int)sb;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#define MICLIP_MXM(IA, IB)                                                                   \
  acc[qi][qj][i][j] =                                                                        \
      TR ? __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[qi][qj][i][j],  \
                                                             0, 0, IB, scb, IA, sca)          \
         : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bf[j], acc[qi][qj][i][j],  \
                                                             0, 0, IA, sca, IB, scb)
        if (j == 0) {
          if (i == 0) MICLIP_MXM(0, 0); else if (i == 1) MICLIP_MXM(1, 0);
          else if (i == 2) MICLIP_MXM(2, 0); else MICLIP_MXM(3, 0);
        } else {
          if (i == 0) MICLIP_MXM(0, 1); else if (i == 1) MICLIP_MXM(1, 1);
          else if (i == 2) MICLIP_MXM(2, 1); else MICLIP_MXM(3, 1);
        }
#undef MICLIP_MXM
      }
    // pin this phase's MFMAs before the next barrier (see lds_barrier_mx)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[qi][qj][i][j]));
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: A0(0)+S(0) B1(0) A1(0) B0(0) A0(1)+S(1) B1(1)
  stage(0, 0);
  stage(3, 0);
  stage(1, 0);
  stage(2, 0);
  if (nk > 1) {
    stage(0, 1);
    stage(3, 1);
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  lds_barrier_mx();
  if (wr == 1) lds_barrier_mx();   // stagger (wave-uniform)
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const char* sA0 = smem + (buf * 4 + 0) * HALF + aoff;
    const char* sA1 = smem + (buf * 4 + 1) * HALF + aoff;
    const char* sB0 = smem + (buf * 4 + 2) * HALF + boff;
    const char* sB1 = smem + (buf * 4 + 3) * HALF + boff;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p == 0 && wr == 0 && t > 0) {
        if (t + 1 < nk)
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (p == 3 && wr == 1 && t + 1 < nk) {
        if (t + 2 < nk)
          asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const int qi = (p >= 2) ? 1 : 0;
      const int qj = (p == 1 || p == 2) ? 1 : 0;
      quadrant(qi ? sA1 : sA0, qj ? sB1 : sB0, p == 0 || p == 2, p != 2);
      if (p == 0) {
        // this K-tile's scales (they arrived with A0(t)). Read from inline asm
        // that also retires them (lgkmcnt(0), which the phase waits for anyway):
        // a plain ds_read here gets a compiler vmcnt(0) in front of it, since
        // hipcc cannot prove the ring disjoint from the in-flight slot DMA.
        const unsigned base = (unsigned)(size_t)(const LDS_AS void*)(smem + SCL + buf * 2048);
        // early-clobber outputs: without "&" hipcc may give the first read's
        // destination the second read's address register (it did: ds_read_b64
        // v[196:197], v196 / ds_read_b32 v207, v197), and whenever the first
        // read's data landed before the second read issued, the W scales came
        // from a garbage address -- a timing-dependent wrong K-tile (seen as
        // run-to-run differences of whole 256-row tiles under two streams)
        u32x2 s2;
        asm volatile(
            "ds_read_b64 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(s2), "=&v"(sb)
            : "v"(base + soa), "v"(base + sob)
            : "memory");
        sa[0] = s2[0];
        sa[1] = s2[1];
      }
      if (p == 0 && t + 1 < nk) stage(1, t + 1);
      if (p == 1 && t + 1 < nk) stage(2, t + 1);
      if (p == 2 && t + 2 < nk) stage(0, t + 2);
      if (p == 3 && t + 2 < nk) stage(3, t + 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_barrier_mx();
      mfma_q(qi, qj);
      lds_barrier_mx();
    }
  }
  if (wr == 0) lds_barrier_mx();   // balance the stagger barrier

  if constexpr (IsEpiStoreH<Epi>::value) {
    // ---- fp16 store from transposed accumulators (gemm.hip gemm256s_kernel's TR
    // store epilogue in one pass of 256 rows): val4 in registers, the 8 output
    // bytes into a row-major fp16 image (pitch 520 B, each row's even and odd 8-B
    // column quads in separate 256-B halves), then per row pair one ds_read_b64 per
    // half and a v_permlane32_swap per dword give each half-wave one whole 512-B
    // row segment to store. The fp16 residual (EpiResidual, c_proj / out-proj):
    // val4 is t = fp16(acc + bias); each lane loads its 16 x pieces (16 B, the
    // readback layout) after staging and adds x + t with packed fp16 adds at
    // readback -- the reference's two roundings, as the fp16 kernels do
    constexpr int TLD = 520;
    char* img = smem;
    lds_barrier_mx();   // every wave is past its last fragment read
    float4 tb[2][2];
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int j = 0; j < 2; ++j) tb[qj][j] = epi.bias4nb(n0 + (wc * 16 + qj * 8 + j * 4 + fk) * 4);
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int qj = 0; qj < 2; ++qj)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int ir = wr * 128 + qi * 64 + i * 16 + fr;
            const int c4 = wc * 16 + qj * 8 + j * 4 + fk;
            const f32x4 a = acc[qi][qj][i][j];
            *(i16x4*)(img + ir * TLD + (c4 & 1) * 256 + (c4 >> 1) * 8) =
                epi.val4(make_float4(a[0], a[1], a[2], a[3]), tb[qj][j]);
          }
    const int h = lane >> 5, li = lane & 31;
    constexpr bool RES = PrefetchX<Epi>::value;
    _Float16* cb;
    int cld;
    if constexpr (RES) {
      cb = epi.X;
      cld = epi.ldx;
    } else {
      cb = epi.C;
      cld = epi.ldc;
    }
    u32x4 xq[16];
    if constexpr (RES) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int row = m0 + wave * 32 + 2 * k + h;
        xq[k] = *(const u32x4*)(cb + (size_t)(row < M ? row : M - 1) * cld + n0 + li * 8);
      }
    }
    lds_barrier_mx();
#pragma unroll
    for (int p0 = 0; p0 < 16; p0 += 2) {
      i16x4 va[2], vb[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int R = wave * 32 + 2 * (p0 + p);
        va[p] = *(const i16x4*)(img + R * TLD + h * 256 + li * 8);
        vb[p] = *(const i16x4*)(img + (R + 1) * TLD + h * 256 + li * 8);
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const u32x2 a = __builtin_bit_cast(u32x2, va[p]), b = __builtin_bit_cast(u32x2, vb[p]);
        const auto s0 = __builtin_amdgcn_permlane32_swap(a[0], b[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(a[1], b[1], false, false);
        u32x4 w = {s0[0], s1[0], s0[1], s1[1]};
        if constexpr (RES) {   // x + t, 8 fp16 pairs of adds
          unsigned t[4] = {w[0], w[1], w[2], w[3]};
          const unsigned x[4] = {xq[p0 + p][0], xq[p0 + p][1], xq[p0 + p][2], xq[p0 + p][3]};
          Epi::template add_x<4>(t, x);
          w = (u32x4){t[0], t[1], t[2], t[3]};
        }
        const int row = m0 + wave * 32 + 2 * (p0 + p) + h;
        if (row < M) *(u32x4*)(cb + (size_t)row * cld + n0 + li * 8) = w;
      }
    }
    return;
  }
  if constexpr (IsEpiMX<Epi>::value) {
    // ---- MX-fp8 epilogue from registers ----
    // Per (qi, qj, i) a lane holds output row lr = wr*128 + qi*64 + i*16 + fr at
    // columns c0 + 4fk .. +3 (j = 0) and c0 + 16 + 4fk .. (j = 1), c0 = wc*64 +
    // qj*32: one 32-column MX block spread over the 4 lanes fr + 16fk. act(acc +
    // bias), block amax over the 8 values and the 4 lanes, E8M0 exponent, 8 e4m3
    // bytes -> an LDS image (pitch 272 B: the 16 rows of a ds_write_b32 group hit
    // distinct 4-bank slots); the tile's 2 KiB of scales -> LDS in the plane's own
    // order ([128-k tile][k-block 4][row & 15][row >> 4 & 15], mx_scale_index).
    // Then whole 256-B rows and 16-B scale pieces go out with dwordx4 stores.
    constexpr int P = 272;
    uint8_t* img = (uint8_t*)smem;
    uint8_t* simg = (uint8_t*)smem + 256 * P;
    lds_barrier_mx();   // every wave is past its last fragment read
    float4 bq[2][2];
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int j = 0; j < 2; ++j) bq[qj][j] = epi.bias4nb(n0 + wc * 64 + qj * 32 + j * 16 + 4 * fk);
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int qj = 0; qj < 2; ++qj)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int lr = wr * 128 + qi * 64 + i * 16 + fr;
          const int c0 = wc * 64 + qj * 32;
          const f32x4 a0 = acc[qi][qj][i][0], a1 = acc[qi][qj][i][1];
          const float4 y0 = Epi::act4(make_float4(a0[0] + bq[qj][0].x, a0[1] + bq[qj][0].y,
                                                  a0[2] + bq[qj][0].z, a0[3] + bq[qj][0].w));
          const float4 y1 = Epi::act4(make_float4(a1[0] + bq[qj][1].x, a1[1] + bq[qj][1].y,
                                                  a1[2] + bq[qj][1].z, a1[3] + bq[qj][1].w));
          float am = fmaxf(fmaxf(fmaxf(fabsf(y0.x), fabsf(y0.y)), fmaxf(fabsf(y0.z), fabsf(y0.w))),
                           fmaxf(fmaxf(fabsf(y1.x), fabsf(y1.y)), fmaxf(fabsf(y1.z), fabsf(y1.w))));
          const int e = mx_exponent(max_rows4(am));
          *(unsigned*)(img + lr * P + c0 + 4 * fk) = mx_pack4(y0, e);
          *(unsigned*)(img + lr * P + c0 + 16 + 4 * fk) = mx_pack4(y1, e);
          if (fk == 0)
            simg[(c0 >> 7) * 1024 + ((c0 >> 5) & 3) * 256 + (lr & 15) * 16 + ((lr >> 4) & 15)] =
                (uint8_t)(e + 127);
        }
    lds_barrier_mx();
    const int ch = tid & 15;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int lr = (tid >> 4) + 32 * k;
      const u32x4 v = *(const u32x4*)(img + lr * P + ch * 16);
      if (m0 + lr < M) *(u32x4*)(epi.C + (size_t)(m0 + lr) * epi.ldc + n0 + ch * 16) = v;
    }
    if (tid < 128)
      *(u32x4*)(epi.S + ((size_t)(m0 >> 8) * epi.kt + (n0 >> 7) + (tid >> 6)) * 1024 +
                (tid & 63) * 16) = *(const u32x4*)(simg + tid * 16);
    return;
  }
  // LDS-staged epilogue (as gemm256_kernel): 2 passes of 128 fp32 rows
  float* stg = (float*)smem;
  const int ec = (tid & 63) * 4;
  const float4 bv = epi.bias4(n0 + ec);
  const bool full = m0 + 256 <= M;
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    lds_barrier_mx();
    i16x4 xr[16];
    if constexpr (PrefetchX<Epi>::value) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int lr = (tid >> 6) + 8 * k;
        const int row = m0 + (lr >> 6) * 128 + qi * 64 + (lr & 63);
        xr[k] = epi.load4(row < M ? row : M - 1, n0 + ec);
      }
    }
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int lr = wr * 64 + i * 16 + fk * 4 + r;
            const int lc = wc * 64 + qj * 32 + j * 16 + fr;
            stg[lr * EPI_LD + lc] = acc[qi][qj][i][j][r];
          }
    lds_barrier_mx();
    if constexpr (PrefetchX<Epi>::value) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int lr = (tid >> 6) + 8 * k;
        const int row = m0 + (lr >> 6) * 128 + qi * 64 + (lr & 63);
        if (full || row < M)
          epi.put4x(row, n0 + ec, *(const float4*)(stg + lr * EPI_LD + ec), bv, xr[k]);
      }
    } else if (full) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int lr = (tid >> 6) + 8 * k;
        const int row = m0 + (lr >> 6) * 128 + qi * 64 + (lr & 63);
        epi.put4(row, n0 + ec, *(const float4*)(stg + lr * EPI_LD + ec), bv);
      }
    } else {
#pragma unroll 4
      for (int k = 0; k < 16; ++k) {
        const int lr = (tid >> 6) + 8 * k;
        const int row = m0 + (lr >> 6) * 128 + qi * 64 + (lr & 63);
        if (row < M) epi.put4(row, n0 + ec, *(const float4*)(stg + lr * EPI_LD + ec), bv);
      }
    }
  }
}

// vmcnt wait at a persistent tile's top: its K-tile 0 (prefetched during the
// previous epilogue) must have landed, while the previous epilogue's S vector
// memory ops and this tile's 5 K-tile-1 ops may stay in flight: vmcnt(S + 5).
MICLIP_DEV void wait_vm_tile_mx(int n) {
  switch (n) {
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Persistent form of gemm256_mx_kernel (the default MX launch): grid = min(tiles,
// CUs), each workgroup walks tiles blockIdx.x + k * grid in the same XCD-grouped
// order, and the next tile's K-tile 0 (its A0 / W1 / A1 / W0 halves and A0's
// scale block) is LDS-DMA'd during this tile's epilogue, as gemm256s_kernel does
// for the fp16 GEMMs (gemm.hip) -- the one-tile-per-workgroup kernel exposes a
// full DMA round trip and the whole epilogue per tile, which at K = 1280 (ViT-H
// QKV, out-proj, c_fc: 10 K-tiles) is a third of the tile's time.
// Same main loop, MFMAs and epilogue arithmetic as gemm256_mx_kernel: outputs
// are bit-identical. LDS: stage buffers [0, 128 KiB); the epilogue image from
// 64 KiB (the buffer-1 half, so buffer 0 can take the prefetch): fp16 outputs in
// two passes of 128 rows (pitch 520 B), MX outputs in one pass (256 x 272 B +
// 2 KiB of scales); then the scale ring (2 x 2 KiB) and the tile's bias (1 KiB,
// DMA'd by wave 0 at the tile's top and retired by the first counted wait).
// Transposed-accumulator epilogues only (fp16 store / fp16 residual / MX out);
// K >= 256 (the tile top assumes a K-tile 1).
template <class Epi>
__global__ __launch_bounds__(512) void gemm256s_mx_kernel(const uint8_t* __restrict__ A,
                                                          const uint8_t* __restrict__ SA,
                                                          const uint8_t* __restrict__ W,
                                                          const uint8_t* __restrict__ SW, int M,
                                                          int N, int K, Epi epi, int gm) {
  static_assert(IsEpiMX<Epi>::value || IsEpiStoreH<Epi>::value, "TR epilogues only");
  constexpr int HALF = 128 * 128;
  constexpr int STG = 4 * HALF;                  // epilogue image (buffer-1 half onward)
  constexpr int TLD = 520;                       // fp16 image pitch
  constexpr int P = 272;                         // MX image pitch
  constexpr int EIMG = IsEpiMX<Epi>::value ? 256 * P + 2048 : 128 * TLD;
  constexpr int SCL = (STG + EIMG + 1023) / 1024 * 1024 > 8 * HALF
                          ? (STG + EIMG + 1023) / 1024 * 1024 : 8 * HALF;
  constexpr int TB = SCL + 4096;
  constexpr int SMEM = TB + 1024;
  static_assert(SMEM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  float4* tbias = (float4*)(smem + TB);

  const int ntn = N / 256, ntm = (M + 255) / 256, ndp = ntm * ntn;
  const int nk = K / 128, KT = nk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int lchunk = (lane & 7) ^ (lane >> 3);
  int m0, n0;
  const uint8_t* asrc[2][2];
  const uint8_t* bsrc[2][2];
  const uint8_t* ssrc;
  auto sources = [&](int id) {
    int tm, tn;
    group_tile(xcd_remap(id, ndp), ntm, ntn, gm, tm, tn);
    m0 = tm * 256;
    n0 = tn * 256;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int sr = (wave * 2 + pp) * 8 + (lane >> 3);
        int ar = m0 + (sr >> 6) * 128 + h * 64 + (sr & 63);
        ar = ar < M ? ar : M - 1;
        asrc[h][pp] = A + (size_t)ar * K + lchunk * 16;
        const int bc = n0 + (sr >> 5) * 64 + h * 32 + (sr & 31);
        bsrc[h][pp] = W + (size_t)bc * K + lchunk * 16;
      }
    ssrc = (wave < 4 ? SA + (size_t)tm * KT * 1024 : SW + (size_t)tn * KT * 1024) +
           (wave & 3) * 256 + lane * 4;
  };
  auto scale_dst = [&](int buf) {
    return smem + SCL + buf * 2048 + (wave >> 2) * 1024 + (wave & 3) * 256;
  };
  auto stage = [&](int slot_kind, int tile) {
    const int buf = tile & 1, k0 = tile * 128;
    char* dst = smem + (buf * 4 + slot_kind) * HALF + wave * 2048;
    const uint8_t* const* src = slot_kind < 2 ? asrc[slot_kind] : bsrc[slot_kind - 2];
    glds16(src[0] + k0, dst);
    glds16(src[1] + k0, dst + 1024);
    if (slot_kind == 0) glds4_hidden(ssrc + (size_t)tile * 1024, scale_dst(buf));
  };
  // the next tile's K-tile 0 in the stage order A0+S, W1, A1, W0 (9 ops per wave),
  // issued from asm (hipcc would otherwise wait for it at the epilogue's LDS reads)
  auto prefetch0 = [&]() {
    const int order[4] = {0, 3, 1, 2};
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int kind = order[o];
      const uint8_t* const* src = kind < 2 ? asrc[kind] : bsrc[kind - 2];
      char* dst = smem + kind * HALF + wave * 2048;
      glds16_hidden(src[0], dst);
      glds16_hidden(src[1], dst + 1024);
      if (kind == 0) glds4_hidden(ssrc, scale_dst(0));
    }
  };
  const int fr = lane & 15, fk = lane >> 4;
  const int aoff = (wr * 64 + fr) * 128, boff = (wc * 32 + fr) * 128;
  const int sw0 = ((0 + fk) ^ (fr & 7)) << 4, sw1 = ((4 + fk) ^ (fr & 7)) << 4;
  const int soa = fk * 256 + fr * 16 + wr * 8, sob = 1024 + fk * 256 + fr * 16 + wc * 4;

  f32x4 acc[2][2][4][2];
  v8i af[4], bf[2];
  unsigned sa[2], sb = 0;
  auto rd8 = [&](const char* p0, const char* p1) {
    const i32x4 lo = *(const i32x4*)p0, hi = *(const i32x4*)p1;
    return (v8i)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto quadrant = [&](const char* sa_, const char* sb_, bool load_a, bool load_b) {
    if (load_a) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = rd8(sa_ + i * 2048 + sw0, sa_ + i * 2048 + sw1);
    }
    if (load_b) {
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = rd8(sb_ + j * 2048 + sw0, sb_ + j * 2048 + sw1);
    }
  };
  // FIRST: K-tile 0's MFMAs start from a zero accumulator (no zeroing v_movs)
  auto mfma_q = [&](int qi, int qj, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    const int sca = qi ? (int)sa[1] : (int)sa[0];
    const int scb = qj ? (int)(sb >> 16) : (int)sb;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 c = FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[qi][qj][i][j];
#define MICLIP_MXM(IA, IB)                                                                      \
  acc[qi][qj][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], c, 0, 0, IB, \
                                                                       scb, IA, sca)
        if (j == 0) {
          if (i == 0) MICLIP_MXM(0, 0); else if (i == 1) MICLIP_MXM(1, 0);
          else if (i == 2) MICLIP_MXM(2, 0); else MICLIP_MXM(3, 0);
        } else {
          if (i == 0) MICLIP_MXM(0, 1); else if (i == 1) MICLIP_MXM(1, 1);
          else if (i == 2) MICLIP_MXM(2, 1); else MICLIP_MXM(3, 1);
        }
#undef MICLIP_MXM
      }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[qi][qj][i][j]));
    __builtin_amdgcn_s_setprio(0);
  };
  auto ktile = [&](int t, auto first_c) {
    const int buf = t & 1;
    const char* sA0 = smem + (buf * 4 + 0) * HALF + aoff;
    const char* sA1 = smem + (buf * 4 + 1) * HALF + aoff;
    const char* sB0 = smem + (buf * 4 + 2) * HALF + boff;
    const char* sB1 = smem + (buf * 4 + 3) * HALF + boff;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p == 0 && wr == 0 && t > 0) {
        if (t + 1 < nk)
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (p == 3 && wr == 1 && t + 1 < nk) {
        if (t + 2 < nk)
          asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const int qi = (p >= 2) ? 1 : 0;
      const int qj = (p == 1 || p == 2) ? 1 : 0;
      quadrant(qi ? sA1 : sA0, qj ? sB1 : sB0, p == 0 || p == 2, p != 2);
      if (p == 0) {
        // the K-tile's scales (gemm256_mx_kernel: early-clobber asm reads)
        const unsigned base = (unsigned)(size_t)(const LDS_AS void*)(smem + SCL + buf * 2048);
        u32x2 s2;
        asm volatile(
            "ds_read_b64 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(s2), "=&v"(sb)
            : "v"(base + soa), "v"(base + sob)
            : "memory");
        sa[0] = s2[0];
        sa[1] = s2[1];
      }
      if (p == 0 && t + 1 < nk) stage(1, t + 1);
      if (p == 1 && t + 1 < nk) stage(2, t + 1);
      if (p == 2 && t + 2 < nk) stage(0, t + 2);
      if (p == 3 && t + 2 < nk) stage(3, t + 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_barrier_mx();
      mfma_q(qi, qj, first_c);
      lds_barrier_mx();
    }
  };

  int prev = -1;   // VMEM ops of the previous epilogue after its prefetch (-1: first tile)
  int id = blockIdx.x;
  if (id < ndp) sources(id);
  for (; id < ndp; id += gridDim.x) {
    if (wave == 0) {
      // the lane index recomputed here (v_mbcnt, opaque to hipcc): a hoisted
      // lane-derived address gets spilled, and its reload's vmcnt(0) would drain
      // the previous epilogue's stores and the prefetch at every tile's top
      int lo;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lo));
      if (epi.bias) {
        glds16_hidden(epi.bias + n0 + lo * 4, tbias);
      } else {
        float z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        tbias[lo] = make_float4(z, z, z, z);
      }
    }
    if (prev < 0) {
      stage(0, 0);
      stage(3, 0);
      stage(1, 0);
      stage(2, 0);
      stage(0, 1);
      stage(3, 1);
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      stage(0, 1);
      stage(3, 1);
      wait_vm_tile_mx(prev + 5);
    }
    lds_barrier_mx();
    if (wr == 1) lds_barrier_mx();   // stagger (wave-uniform)
    ktile(0, std::true_type{});
    for (int t = 1; t < nk; ++t) ktile(t, std::false_type{});
    if (wr == 0) lds_barrier_mx();   // balance the stagger barrier
    lds_barrier_mx();                // every wave is done with both buffers
    const int cm0 = m0, cn0 = n0;
    const bool full = cm0 + 256 <= M;
    const int nid = id + gridDim.x;
    // lane-derived epilogue offsets from a lane index recomputed per tile (see the
    // bias DMA above): hoisted out of the tile loop they are spilled around it
    int el;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(el));
    const int efr = el & 15, efk = el >> 4, etid = wave * 64 + el;
    float4 tb[2][2];
#pragma unroll
    for (int qj = 0; qj < 2; ++qj)
#pragma unroll
      for (int j = 0; j < 2; ++j) tb[qj][j] = tbias[wc * 16 + qj * 8 + j * 4 + efk];
    if constexpr (IsEpiStoreH<Epi>::value) {
      // fp16 store / residual: gemm256s_kernel's transposed-accumulator epilogue
      // (two passes of 128 rows; each half-wave stores one 512-B row segment)
      char* img = smem + STG;
      constexpr bool RES = PrefetchX<Epi>::value;
      _Float16* cb;
      int cld;
      if constexpr (RES) {
        cb = epi.X;
        cld = epi.ldx;
      } else {
        cb = epi.C;
        cld = epi.ldc;
      }
      const int h = el >> 5, li = el & 31;
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        if (qi > 0) lds_barrier_mx();   // pass 0's readers are done with the image
        u32x4 xq[8];
        if constexpr (RES) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int ir = wave * 16 + 2 * k + h;
            const int row = cm0 + (ir >> 6) * 128 + qi * 64 + (ir & 63);
            xq[k] = *(const u32x4*)(cb + (size_t)(row < M ? row : M - 1) * cld + cn0 + li * 8);
          }
        }
#pragma unroll
        for (int qj = 0; qj < 2; ++qj)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int ir = wr * 64 + i * 16 + efr;
              const int c4 = wc * 16 + qj * 8 + j * 4 + efk;
              const f32x4 a = acc[qi][qj][i][j];
              *(i16x4*)(img + ir * TLD + (c4 & 1) * 256 + (c4 >> 1) * 8) =
                  epi.val4(make_float4(a[0], a[1], a[2], a[3]), tb[qj][j]);
            }
        if (qi == 0) {
          if constexpr (RES) {
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(xq[k]));
          }
          if (nid < ndp) {   // the next tile's sources only now (not live across the math)
            sources(nid);
            prefetch0();
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lds_barrier_mx();
#pragma unroll
        for (int p0 = 0; p0 < 8; p0 += 2) {
          i16x4 va[2], vb[2];
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const int R = wave * 16 + 2 * (p0 + p);
            va[p] = *(const i16x4*)(img + R * TLD + h * 256 + li * 8);
            vb[p] = *(const i16x4*)(img + (R + 1) * TLD + h * 256 + li * 8);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(va[0]), "+v"(va[1]), "+v"(vb[0]), "+v"(vb[1]));
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const u32x2 a = __builtin_bit_cast(u32x2, va[p]), b = __builtin_bit_cast(u32x2, vb[p]);
            const auto s0 = __builtin_amdgcn_permlane32_swap(a[0], b[0], false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(a[1], b[1], false, false);
            u32x4 w = {s0[0], s1[0], s0[1], s1[1]};
            if constexpr (RES) {
              unsigned t[4] = {w[0], w[1], w[2], w[3]};
              const unsigned x[4] = {xq[p0 + p][0], xq[p0 + p][1], xq[p0 + p][2], xq[p0 + p][3]};
              Epi::template add_x<4>(t, x);
              w = (u32x4){t[0], t[1], t[2], t[3]};
            }
            const int ir = wave * 16 + 2 * (p0 + p) + h;
            const int row = cm0 + (ir >> 6) * 128 + qi * 64 + (ir & 63);
            if (full || row < M) *(u32x4*)(cb + (size_t)row * cld + cn0 + li * 8) = w;
          }
        }
      }
      // after the prefetch: pass 0's 8 stores, pass 1's x loads (residual) and 8 stores
      prev = full ? (RES ? 24 : 16) : 0;
    } else {
      // MX-fp8 out (gemm256_mx_kernel's EpiMX epilogue, image at STG)
      uint8_t* img = (uint8_t*)smem + STG;
      uint8_t* simg = img + 256 * P;
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int qj = 0; qj < 2; ++qj)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int lr = wr * 128 + qi * 64 + i * 16 + efr;
            const int c0 = wc * 64 + qj * 32;
            const f32x4 a0 = acc[qi][qj][i][0], a1 = acc[qi][qj][i][1];
            const float4 y0 = Epi::act4(make_float4(a0[0] + tb[qj][0].x, a0[1] + tb[qj][0].y,
                                                    a0[2] + tb[qj][0].z, a0[3] + tb[qj][0].w));
            const float4 y1 = Epi::act4(make_float4(a1[0] + tb[qj][1].x, a1[1] + tb[qj][1].y,
                                                    a1[2] + tb[qj][1].z, a1[3] + tb[qj][1].w));
            float am = fmaxf(fmaxf(fmaxf(fabsf(y0.x), fabsf(y0.y)), fmaxf(fabsf(y0.z), fabsf(y0.w))),
                             fmaxf(fmaxf(fabsf(y1.x), fabsf(y1.y)), fmaxf(fabsf(y1.z), fabsf(y1.w))));
            const int e = mx_exponent(max_rows4(am));
            *(unsigned*)(img + lr * P + c0 + 4 * efk) = mx_pack4(y0, e);
            *(unsigned*)(img + lr * P + c0 + 16 + 4 * efk) = mx_pack4(y1, e);
            if (efk == 0)
              simg[(c0 >> 7) * 1024 + ((c0 >> 5) & 3) * 256 + (lr & 15) * 16 + ((lr >> 4) & 15)] =
                  (uint8_t)(e + 127);
          }
      if (nid < ndp) {
        sources(nid);
        prefetch0();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_barrier_mx();
      const int ch = etid & 15;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int lr = (etid >> 4) + 32 * k;
        const u32x4 v = *(const u32x4*)(img + lr * P + ch * 16);
        if (full || cm0 + lr < M)
          *(u32x4*)(epi.C + (size_t)(cm0 + lr) * epi.ldc + cn0 + ch * 16) = v;
      }
      if (etid < 128)
        *(u32x4*)(epi.S + ((size_t)(cm0 >> 8) * epi.kt + (cn0 >> 7) + (etid >> 6)) * 1024 +
                  (etid & 63) * 16) = *(const u32x4*)(simg + etid * 16);
      prev = full ? (wave < 2 ? 9 : 8) : 0;
    }
    lds_barrier_mx();   // the image is free for the next tile's epilogue
  }
}

// Rows of fp32 / fp16 -> MX-fp8 (data + tiled scales). One wave per 256
// consecutive k of one row (8 blocks of 32, 4 elements per lane).
template <typename TI>
__global__ __launch_bounds__(256) void quant_mx_kernel(const TI* __restrict__ in, int R, int K,
                                                       uint8_t* __restrict__ q,
                                                       uint8_t* __restrict__ sc) {
  const int lane = threadIdx.x & 63;
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);   // (row, 256-k segment)
  const int nseg = K / 256;
  const int r = seg / nseg, k = (seg - r * nseg) * 256 + 4 * lane;
  if (r >= R) return;
  float4 v;
  if constexpr (std::is_same_v<TI, float>) {
    v = *(const float4*)(in + (size_t)r * K + k);
  } else {
    const i16x4 h = *(const i16x4*)(in + (size_t)r * K + k);
    v = make_float4(from_bits<TI>(h[0]), from_bits<TI>(h[1]), from_bits<TI>(h[2]),
                    from_bits<TI>(h[3]));
  }
  int e;
  const unsigned w = mx_quant4(v, e);
  *(unsigned*)(q + (size_t)r * K + k) = w;
  if ((lane & 7) == 0) sc[mx_scale_index(r, k >> 5, K / 128)] = (uint8_t)(e + 127);
}

// fp16 rows -> MX-fp8, 16-B loads: a lane takes 8 consecutive k, a 32-block is a
// quad (max by two DPP steps), one chunk per thread (2 per thread: 0.107 vs 0.103 ms
// at C5's 131 584 x 1280, 4: 0.112; profiles/r05/quant_mx/). R * K / 8 is a multiple
// of 4, so a quad is either wholly in range or wholly past the end.
__global__ __launch_bounds__(256) void quant_mx_h8_kernel(const _Float16* __restrict__ in,
                                                          size_t chunks, int K,
                                                          uint8_t* __restrict__ q,
                                                          uint8_t* __restrict__ sc) {
  const int kc = K / 8;
  {
    const size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
    const bool valid = c < chunks;
    const i16x8 h = *(const i16x8*)(in + (valid ? c : 0) * 8);
    float y[8];
    float a = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      y[e] = from_bits<_Float16>(h[e]);
      a = fmaxf(a, fabsf(y[e]));
    }
    a = fmaxf(a, dppf<0xB1>(a));   // quad_perm [1,0,3,2]
    a = fmaxf(a, dppf<0x4E>(a));   // quad_perm [2,3,0,1]
    const int ex = mx_exponent(a);
    const unsigned lo = mx_pack4(make_float4(y[0], y[1], y[2], y[3]), ex);
    const unsigned hi = mx_pack4(make_float4(y[4], y[5], y[6], y[7]), ex);
    if (valid) {
      *(uint2*)(q + c * 8) = make_uint2(lo, hi);
      if ((threadIdx.x & 3) == 0) {
        // 32-bit index math (chunks < 2^31, checked by the launcher)
        const unsigned cu = (unsigned)c, r = cu / (unsigned)kc;
        const int k = (int)(cu - r * (unsigned)kc) * 8;
        sc[mx_scale_index((int)r, k >> 5, K / 128)] = (uint8_t)(ex + 127);
      }
    }
  }
}

int cu_count() {
  static int ncu = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return ncu;
}

// variant 0: the persistent kernel where it applies (K >= 256), else one tile per
// workgroup; 1: one tile per workgroup (gemm256_mx_kernel); 2: persistent (refused
// where it does not apply). All bit-identical.
template <class Epi>
hipError_t launch_mx(const void* A, const void* SA, const void* W, const void* SW, int M, int N,
                     int K, Epi epi, hipStream_t s, int variant) {
  if (M < 1 || N % 256 || K % 128 || K < 128) return hipErrorInvalidValue;
  if (variant < 0 || variant > 2) return hipErrorInvalidValue;
  const int tiles = (M + 255) / 256 * (N / 256);
  const int gm = 4;   // tile-row group (r03 sweep: 4 and 2 tie, 8 -1 %, 16 -2.7 %)
  if constexpr (IsEpiMX<Epi>::value || IsEpiStoreH<Epi>::value) {
    if (variant != 1 && K >= 256) {
      const int ncu = cu_count();
      hipLaunchKernelGGL((gemm256s_mx_kernel<Epi>), dim3(tiles < ncu ? tiles : ncu), dim3(512), 0,
                         s, (const uint8_t*)A, (const uint8_t*)SA, (const uint8_t*)W,
                         (const uint8_t*)SW, M, N, K, epi, gm);
      return hipGetLastError();
    }
  }
  if (variant == 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm256_mx_kernel<Epi>), dim3(tiles), dim3(512), 0, s, (const uint8_t*)A,
                     (const uint8_t*)SA, (const uint8_t*)W, (const uint8_t*)SW, M, N, K, epi, gm);
  return hipGetLastError();
}

}  // namespace

size_t mx_scale_bytes(int rows, int K) { return (size_t)((rows + 255) / 256) * (K / 128) * 1024; }

hipError_t quant_mx(int in_f16, const void* in, int R, int K, void* q, void* sc, hipStream_t s) {
  if (R < 1 || K % 256) return hipErrorInvalidValue;
  const int segs = R * (K / 256);
  // in_f16: 0 fp32, 1 fp16 (16-B loads, lane-quad blocks), 2 fp16 through the
  // older 8-lane-block kernel (op level only: the byte-identity test)
  if (in_f16 == 1) {
    const size_t chunks = (size_t)R * (K / 8);
    if (chunks >= ((size_t)1 << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(quant_mx_h8_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s,
                       (const _Float16*)in, chunks, K, (uint8_t*)q, (uint8_t*)sc);
  } else if (in_f16)
    hipLaunchKernelGGL(quant_mx_kernel<_Float16>, dim3((segs + 3) / 4), dim3(256), 0, s,
                       (const _Float16*)in, R, K, (uint8_t*)q, (uint8_t*)sc);
  else
    hipLaunchKernelGGL(quant_mx_kernel<float>, dim3((segs + 3) / 4), dim3(256), 0, s,
                       (const float*)in, R, K, (uint8_t*)q, (uint8_t*)sc);
  return hipGetLastError();
}

hipError_t gemm_mx(const void* A, const void* SA, const void* W, const void* SW, const float* bias,
                   void* C, void* CS, int M, int N, int K, int epi, int act, hipStream_t s,
                   int variant) {
  if (!A || !SA || !W || !SW || !C) return hipErrorInvalidValue;
  switch (epi) {
    case 0:   // fp16 store: act(acc + bias)
      if (act == ACT_NONE)
        return launch_mx(A, SA, W, SW, M, N, K, EpiStore<_Float16, ACT_NONE>{(_Float16*)C, bias, N}, s, variant);
      if (act == ACT_QUICKGELU)
        return launch_mx(A, SA, W, SW, M, N, K,
                         EpiStore<_Float16, ACT_QUICKGELU>{(_Float16*)C, bias, N}, s, variant);
      return launch_mx(A, SA, W, SW, M, N, K, EpiStore<_Float16, ACT_GELU>{(_Float16*)C, bias, N}, s, variant);
    case 1:   // fp16 residual stream += acc + bias
      if (!bias) return hipErrorInvalidValue;
      return launch_mx(A, SA, W, SW, M, N, K, EpiResidual<_Float16>{(_Float16*)C, bias, N}, s, variant);
    case 5:   // MX-fp8 out (data C [M, N] bytes + scale plane CS): act(acc + bias)
      if (!CS || N % 128) return hipErrorInvalidValue;
      if (act == ACT_QUICKGELU)
        return launch_mx(A, SA, W, SW, M, N, K,
                         EpiMX<ACT_QUICKGELU>{(uint8_t*)C, (uint8_t*)CS, bias, N, N / 128}, s, variant);
      if (act == ACT_GELU)
        return launch_mx(A, SA, W, SW, M, N, K,
                         EpiMX<ACT_GELU>{(uint8_t*)C, (uint8_t*)CS, bias, N, N / 128}, s, variant);
      if (act == ACT_GELU_TANH)
        return launch_mx(A, SA, W, SW, M, N, K,
                         EpiMX<ACT_GELU_TANH>{(uint8_t*)C, (uint8_t*)CS, bias, N, N / 128}, s, variant);
      return launch_mx(A, SA, W, SW, M, N, K,
                       EpiMX<ACT_NONE>{(uint8_t*)C, (uint8_t*)CS, bias, N, N / 128}, s, variant);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace miclip
