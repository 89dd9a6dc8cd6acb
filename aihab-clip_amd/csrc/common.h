// Shared device helpers for the miclip CDNA4 (gfx950) kernels.
//
// Compute dtype T is either _Float16 (the reference's GPU precision:
// convert_weights, clip/model.py:372-393) or __bf16. Both run on the same
// MFMA rate on gfx950; accumulation, LayerNorm statistics, softmax and the
// residual stream are fp32 everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define MICLIP_DEV __device__ __forceinline__

// In-kernel cycle stamps, compiled only into the diagnostic programs of
// scripts/stamps/ (which define MICLIP_STAMPS before including a kernel source);
// in the library every macro is empty. Per wave: the s_memtime cycles spent in
// up to 8 segments (wave-uniform, SGPRs: s_memtime is a scalar READ), and at
// exit lane 0 stores {segments, total cycles, s_memrealtime ticks (100 MHz)}
// to miclip_stamp_buf[slot] with ordinary vector stores.
#ifdef MICLIP_STAMPS
constexpr int kStampWords = 10;
extern __device__ unsigned long long miclip_stamp_buf[];
struct StampAcc {
  unsigned long long t, t0, r0, a0, a1, a2, a3, a4, a5, a6, a7;
};
#define MICLIP_STAMP_BEGIN                                                             \
  StampAcc st_;                                                                        \
  st_.r0 = __builtin_amdgcn_s_memrealtime();                                           \
  st_.t = st_.t0 = __builtin_amdgcn_s_memtime();                                       \
  st_.a0 = st_.a1 = st_.a2 = st_.a3 = st_.a4 = st_.a5 = st_.a6 = st_.a7 = 0
#define MICLIP_STAMP(i)                                                                \
  do {                                                                                 \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                        \
    st_.a##i += n_ - st_.t;                                                            \
    st_.t = n_;                                                                        \
  } while (0)
#define MICLIP_STAMP_END(slot)                                                         \
  do {                                                                                 \
    const unsigned long long e_ = __builtin_amdgcn_s_memtime();                        \
    const unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                    \
    if ((threadIdx.x & 63) == 0) {                                                     \
      unsigned long long* p_ = miclip_stamp_buf + (size_t)(slot) * kStampWords;        \
      p_[0] = st_.a0; p_[1] = st_.a1; p_[2] = st_.a2; p_[3] = st_.a3;                  \
      p_[4] = st_.a4; p_[5] = st_.a5; p_[6] = st_.a6; p_[7] = st_.a7;                  \
      p_[8] = e_ - st_.t0; p_[9] = r_ - st_.r0;                                        \
    }                                                                                  \
  } while (0)
#else
#define MICLIP_STAMP_BEGIN
#define MICLIP_STAMP(i)
#define MICLIP_STAMP_END(slot)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4_vs __attribute__((__vector_size__(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Tiled MX scale planes (gemm_mx.hip): E8M0 byte of (row r, 32-k block kb) of an
// operand with KT = K / 128 K-tiles -- per (256-row block, K-tile) one 1-KiB block
// [kb & 3][r & 15][(r >> 4) & 15], the order the fp8 GEMM's lanes read.
__host__ __device__ inline size_t mx_scale_index(int r, int kb, int KT) {
  return ((size_t)(r >> 8) * KT + (kb >> 2)) * 1024 + (kb & 3) * 256 + (r & 15) * 16 +
         ((r >> 4) & 15);
}

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

namespace miclip {

enum DType { kF16 = 0, kBF16 = 1 };
// image input element type of encode_image_ex (MICLIP_F32 in include/miclip.h)
constexpr int kIn32 = 3;

template <typename T> struct Mfma;

template <> struct Mfma<_Float16> {
  typedef f16x8 v8;
  static MICLIP_DEV f32x4 m16(const i16x8& a, const i16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
  static MICLIP_DEV f32x16 m32(const i16x8& a, const i16x8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

template <> struct Mfma<__bf16> {
  typedef bf16x8 v8;
  static MICLIP_DEV f32x4 m16(const i16x8& a, const i16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
  static MICLIP_DEV f32x16 m32(const i16x8& a, const i16x8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

// float <-> storage type (round to nearest even; the compiler emits v_cvt_pk_*)
template <typename T> MICLIP_DEV T to_t(float x) { return static_cast<T>(x); }
template <typename T> MICLIP_DEV float to_f(T x) { return static_cast<float>(x); }
template <typename T> MICLIP_DEV short to_bits(float x) {
  return __builtin_bit_cast(short, static_cast<T>(x));
}
template <typename T> MICLIP_DEV float from_bits(short b) {
  return static_cast<float>(__builtin_bit_cast(T, b));
}

MICLIP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// DPP lane move within a 16-lane row (bound_ctrl: lanes with no source read 0)
template <int CTRL>
MICLIP_DEV float dppf(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}

// Sum over the 32 lanes of a half-wave: DPP (quad_perm, row_half_mirror,
// row_mirror) within each 16-lane row, then v_permlane16_swap (rows 0<->1,
// 2<->3) for the last step -- no LDS round trip; every lane of the half gets the
// same value (row 0's + row 1's partial, in that order, on both rows).
MICLIP_DEV float half_sum(float x) {
  x += dppf<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dppf<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dppf<0x141>(x);   // row_half_mirror (lane i <-> 7-i of its 8)
  x += dppf<0x140>(x);   // row_mirror (lane i <-> 15-i of its 16)
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}

MICLIP_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 16-byte async global -> LDS copy (global_load_lds_dwordx4). LDS destination is
// the wave-uniform `lds` base + lane*16; the global source is per lane.
MICLIP_DEV void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)g, (LDS_AS void*)lds, 16, 0, 0);
}

// Same DMA, issued from inline asm so hipcc's waitcnt pass does not see it:
// hipcc then never waits vmcnt(0) for it before an unrelated ds_read or load
// (it cannot prove the LDS ranges disjoint). The caller retires it with its
// own `s_waitcnt vmcnt` + barrier. `lds` must be wave-uniform.
// 4-B form (each lane one dword, 256 B per wave): per-lane clamped sources at
// row granularity (the persistent GEMM's row statistics).
MICLIP_DEV void glds4_hidden(const void* g, const void* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(const LDS_AS void*)lds);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(dst)
      : "memory");
}

MICLIP_DEV void glds16_hidden(const void* g, const void* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(const LDS_AS void*)lds);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(dst)
      : "memory");
}

// The same DMA through a buffer resource (hidden from hipcc's waitcnt pass like
// glds16_hidden): `desc` is a raw buffer descriptor in SGPRs (make_buffer_desc),
// `voff` a per-lane 32-bit byte offset -- one VGPR per source instead of a 64-bit
// address per piece. `lds` must be wave-uniform.
typedef unsigned int u32x4s __attribute__((ext_vector_type(4)));
MICLIP_DEV u32x4s make_buffer_desc(const void* base) {
  const unsigned long long a = (unsigned long long)base;
  u32x4s d = {(unsigned)a, (unsigned)(a >> 32) & 0xffffu, 0x7fffffffu, 0x00020000u};
  d[0] = __builtin_amdgcn_readfirstlane(d[0]);
  d[1] = __builtin_amdgcn_readfirstlane(d[1]);
  return d;
}
MICLIP_DEV void blds16_hidden(u32x4s desc, unsigned voff, const void* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(const LDS_AS void*)lds);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(desc), "s"(dst)
      : "memory");
}

// Grouped tile order: consecutive ids walk `gm` tile-rows column by column, so
// the tiles one XCD runs together share A panels and W panels in its L2
// (ids are already XCD-contiguous after xcd_remap). gm <= 1: row-major.
MICLIP_DEV void group_tile(int id, int ntm, int ntn, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = id / ntn;
    tn = id - tm * ntn;
    return;
  }
  const int per = gm * ntn, g = id / per, first = g * gm;
  const int rows = ntm - first < gm ? ntm - first : gm;
  const int idx = id - g * per;
  tm = first + idx % rows;
  tn = idx / rows;
}

MICLIP_DEV i16x4 ds_read_tr16_b64(const void* lds) {
  return __builtin_bit_cast(
      i16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_vs*)(lds)));
}
MICLIP_DEV i16x4 ds_read_tr16_b64(const LDS_AS char* lds) {
  return __builtin_bit_cast(
      i16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_vs*)(lds)));
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5.5 T1): blocks that
// the dispatcher deals to one XCD (b, b+8, ...) get a contiguous range of tiles.
MICLIP_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

}  // namespace miclip
