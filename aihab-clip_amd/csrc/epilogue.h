// GEMM epilogue functors and their helpers, shared by the f16/bf16 GEMMs
// (gemm.hip) and the MX-fp8 GEMM (gemm_mx.hip). Internal to the library.
#pragma once
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace miclip {

namespace {

// Stores issued from inline asm are invisible to hipcc's waitcnt pass. The
// register epilogue of the persistent GEMM uses them: a compiler-visible store
// inside the K-tile loop makes hipcc wait vmcnt(0) at the loop header (before
// the next K-tile's ds_reads reuse the data registers), which would drain the
// next tile's in-flight LDS-DMA every K-tile. `s_nop 1` closes the statement so
// the data registers are read before anything overwrites them.
MICLIP_DEV void st_b64_asm(void* p, i16x4 v) {
  asm volatile("global_store_dwordx2 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
MICLIP_DEV void st_b128_asm(void* p, float4 v) {
  const f32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}

// Epilogue functors. The kernels hoist the per-column bias load (`bias4` /
// `bias1`, once per column a thread owns) and then call `put4` (4 consecutive
// columns of one row, 16-B aligned) or `put1` with the raw fp32 accumulator.
MICLIP_DEV float4 ld_bias4(const float* b, int col) {
  return b ? *(const float4*)(b + col) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Branch-free form for the register epilogue: a null bias becomes a buffer
// descriptor with zero records, whose loads return 0 (a `b ? load : 0` select
// makes hipcc branch around the load and wait vmcnt(0) at the join).
MICLIP_DEV float4 ld_bias4_nb(const float* b, int col) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, b ? 0x7fffffff : 0, 0x00020000);
  const f32x4 v = __builtin_bit_cast(
      f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)col * 4u, 0, 0));
  return make_float4(v[0], v[1], v[2], v[3]);
}

// Exact GELU, 0.5 v erfc(-v/sqrt2), for the open_clip ViT-H/14 MLP (nn.GELU).
// erfc from the Chebyshev fit of Numerical Recipes' erfcc (fractional error
// < 1.2e-7 over the whole line), rewritten for the hardware: base-2 exponent
// (v_exp_f32) with log2(e) folded into the coefficients, the 0.5 folded into
// the exponent, and erfc(-z) = 2 - erfc(z) for v >= 0. 19 VALU ops against
// ~40 for libm erff, and no 1 + erf cancellation in the negative tail (CPU
// check: max abs error 2.4e-7, max rel 5e-6 against double erfc on [-12, 12]).
// Every step is an explicit mul / fma so the scalar and the packed form
// below round identically (the tile and tail paths must agree bit for bit).
namespace gelu_nr {
constexpr float L = 1.4426950408889634f;
constexpr float kT = 0.35355339059327373f;  // 0.5 / sqrt(2): t = 1 / (1 + z/2)
constexpr float kC[10] = {0.17087277f * L,  -0.82215223f * L, 1.48851587f * L,
                          -1.13520398f * L, 0.27886807f * L,  -0.18628806f * L,
                          0.09678418f * L,  0.37409196f * L,  1.00002368f * L,
                          -1.26551223f * L - 1.0f};
constexpr float kQ = -0.5f * L;              // -z^2 log2(e) = v^2 * kQ
}  // namespace gelu_nr

MICLIP_DEV float gelu_erf(float v) {
  using namespace gelu_nr;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_fabsf(v), kT, 1.0f));
  float p = kC[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) p = __builtin_fmaf(t, p, kC[i]);
  const float vt = v * t;
  const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(v * v, kQ, p));
  const float hv = vt * e;                         // 0.5 v erfc(|v|/sqrt2)
  const float pos = __builtin_fmaf(-vt, e, v);     // v - hv
  return v >= 0.f ? pos : hv;
}

MICLIP_DEV f32x2 gelu_erf2(f32x2 v) {
  using namespace gelu_nr;
  const f32x2 a = {__builtin_fabsf(v[0]), __builtin_fabsf(v[1])};
  const f32x2 d = __builtin_elementwise_fma(a, (f32x2){kT, kT}, (f32x2){1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = {kC[0], kC[0]};
#pragma unroll
  for (int i = 1; i < 10; ++i) p = __builtin_elementwise_fma(t, p, (f32x2){kC[i], kC[i]});
  const f32x2 vt = v * t;
  const f32x2 x = __builtin_elementwise_fma(v * v, (f32x2){kQ, kQ}, p);
  const f32x2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
  const f32x2 hv = vt * e;
  const f32x2 pos = __builtin_elementwise_fma(-vt, e, v);
  return (f32x2){v[0] >= 0.f ? pos[0] : hv[0], v[1] >= 0.f ? pos[1] : hv[1]};
}

constexpr float kQuickGeluK = -1.702f * 1.4426950408889634f;

// GELU, tanh form: x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)) on two values,
// base 2 with log2(e) folded: t = x (a + b x^2), y = x / (1 + 2^t). Large |x|
// saturates cleanly (2^t -> inf gives -0, 2^t -> 0 gives x). 2 transcendentals +
// 5 packed ops per pair against the erf fit's 2 + ~14.
constexpr float kGeluTanhA = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
constexpr float kGeluTanhB = kGeluTanhA * 0.044715f;
MICLIP_DEV f32x2 gelu_tanh2(f32x2 v) {
  const f32x2 p = __builtin_elementwise_fma(v * v, (f32x2){kGeluTanhB, kGeluTanhB},
                                            (f32x2){kGeluTanhA, kGeluTanhA});
  const f32x2 t = v * p;
  const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])} +
                  (f32x2){1.0f, 1.0f};
  return v * (f32x2){__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}

// QuickGELU on two values with packed fp32 mul / add (v_pk_mul_f32, v_pk_add_f32):
// the c_fc epilogue is VALU-bound, and these round exactly like the scalar form.
MICLIP_DEV f32x2 quick_gelu2(f32x2 v) {
  const f32x2 t = v * (f32x2){kQuickGeluK, kQuickGeluK};
  const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])} +
                  (f32x2){1.0f, 1.0f};
  return v * (f32x2){__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}

template <int ACT>
MICLIP_DEV float act_fn(float v) {
  // x * sigmoid(1.702 x) (clip/model.py:160-162): one mul into v_exp (base 2,
  // -1.702 log2 e folded), v_rcp, no IEEE divide; same op sequence as the
  // packed quick_gelu2 below
  if (ACT == ACT_QUICKGELU)
    return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * kQuickGeluK));
  if (ACT == ACT_GELU) return gelu_erf(v);
  return v;
}

// The activation is a template parameter so that the QKV projection (no
// activation) and the MLP c_fc (QuickGELU) are distinct kernels in a profile.
template <typename T, int ACT>
struct EpiStore {
  T* C;
  const float* bias;
  int ldc;
  int nt = 0;   // non-temporal output stores (gemm.hip gemm_nt(): off, measured level)
  MICLIP_DEV float4 bias4(int col) const { return ld_bias4(bias, col); }
  MICLIP_DEV float4 bias4nb(int col) const { return ld_bias4_nb(bias, col); }
  MICLIP_DEV float bias1(int col) const { return bias ? bias[col] : 0.f; }
  // The fp32 result is pinned in a register before the conversion: otherwise
  // hipcc may fuse the last multiply (or add) with the conversion into one
  // v_fma_mix* (a single rounding) in some call sites and not in others, and
  // the tile and tail paths would differ in the last bit. Not `volatile`: an
  // opaque op is enough to stop the fusion, and a volatile one would also pin
  // the ORDER of all the epilogue's pins, serialising the rows' dependent
  // exp -> rcp -> mul chains instead of interleaving them.
  MICLIP_DEV static float fin(float y) {
    asm("" : "+v"(y));
    return y;
  }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4 b) const {
    const i16x4 o = val4(v, b);
    if constexpr (ASM)
      st_b64_asm(C + (size_t)r * ldc + c, o);
    else if (nt)
      __builtin_nontemporal_store(o, (i16x4*)(C + (size_t)r * ldc + c));
    else
      *(i16x4*)(C + (size_t)r * ldc + c) = o;
  }
  // the 4 output elements of put4, returned instead of stored (the persistent
  // kernel's transposed-accumulator epilogue stages them in LDS)
  MICLIP_DEV i16x4 val4(float4 v, float4 b) const {
    i16x4 o;
    if constexpr (ACT == ACT_GELU || ACT == ACT_QUICKGELU) {  // packed-fp32 forms, same rounding
      const f32x2 y0 = (f32x2){v.x, v.y} + (f32x2){b.x, b.y};
      const f32x2 y1 = (f32x2){v.z, v.w} + (f32x2){b.z, b.w};
      const f32x2 lo = ACT == ACT_GELU ? gelu_erf2(y0) : quick_gelu2(y0);
      const f32x2 hi = ACT == ACT_GELU ? gelu_erf2(y1) : quick_gelu2(y1);
      o[0] = to_bits<T>(fin(lo[0]));
      o[1] = to_bits<T>(fin(lo[1]));
      o[2] = to_bits<T>(fin(hi[0]));
      o[3] = to_bits<T>(fin(hi[1]));
    } else {
      // packed adds (v_pk_add_f32), the same rounding as the scalar form of put1
      f32x2 y0 = (f32x2){v.x, v.y} + (f32x2){b.x, b.y};
      f32x2 y1 = (f32x2){v.z, v.w} + (f32x2){b.z, b.w};
      asm("" : "+v"(y0), "+v"(y1));
      o[0] = to_bits<T>(y0[0]);
      o[1] = to_bits<T>(y0[1]);
      o[2] = to_bits<T>(y1[0]);
      o[3] = to_bits<T>(y1[1]);
    }
    return o;
  }
  MICLIP_DEV void put1(int r, int c, float v, float b) const {
    C[(size_t)r * ldc + c] = to_t<T>(fin(act_fn<ACT>(v + b)));
  }
};

// LayerNorm folded into the projection that consumes it (ln_1 -> QKV, ln_2 ->
// c_fc; clip/model.py:184-185). With n = (x - mu) * rs the normalised row,
//   LN(x) . W^T + b = rs * (x . W'^T - mu * s) + c,
//   W' = W diag(gamma) (compute dtype), s_j = sum_k W'_jk, c_j = b_j + sum_k beta_k W_jk,
// so the GEMM reads the fp16 residual stream x directly and the normalised
// activations h are never written or re-read. Per row {mu, rs} comes from
// ln_stats (norm.hip: the LayerNorm kernel's own two-pass statistics); s and c
// are built once per weight load (ln_fold). `bias` holds c. The persistent
// kernel stages each tile's 256 row statistics in LDS and calls put4ln; the
// other kernels call put4 / put1, which load them here. Same float expression
// on every path (pinned by fin), so the tile and tail paths agree bit for bit.
template <typename T, int ACT>
struct EpiStoreLN {
  T* C;
  const float* bias;     // c
  const float* colsum;   // s
  const float2* stats;   // [M] {mu, rs}
  int ldc;
  MICLIP_DEV float4 bias4(int col) const { return ld_bias4(bias, col); }
  MICLIP_DEV float4 bias4nb(int col) const { return ld_bias4_nb(bias, col); }
  MICLIP_DEV float bias1(int col) const { return bias[col]; }
  MICLIP_DEV float4 colsum4nb(int col) const { return ld_bias4_nb(colsum, col); }
  MICLIP_DEV static float fin(float y) {
    asm("" : "+v"(y));
    return y;
  }
  MICLIP_DEV static float z(float v, float s, float2 st, float c) {
    return fin(__builtin_fmaf(st.y, __builtin_fmaf(-st.x, s, v), c));
  }
  // two columns at once: the same two fused multiply-adds per element as z(),
  // issued as packed v_pk_fma_f32 (same rounding), so tile and tail paths agree
  MICLIP_DEV static f32x2 z2(f32x2 v, f32x2 s, float2 st, f32x2 c) {
    const f32x2 t = __builtin_elementwise_fma((f32x2){-st.x, -st.x}, s, v);
    f32x2 y = __builtin_elementwise_fma((f32x2){st.y, st.y}, t, c);
    asm("" : "+v"(y));
    return y;
  }
  template <bool ASM = false>
  MICLIP_DEV void put4ln(int r, int c, float4 v, float4 b, float4 s, float2 st) const {
    const i16x4 o = val4ln(v, b, s, st);
    if constexpr (ASM)
      st_b64_asm(C + (size_t)r * ldc + c, o);
    else
      *(i16x4*)(C + (size_t)r * ldc + c) = o;
  }
  // put4ln's 4 output elements, returned instead of stored
  MICLIP_DEV i16x4 val4ln(float4 v, float4 b, float4 s, float2 st) const {
    const f32x2 y0 = z2((f32x2){v.x, v.y}, (f32x2){s.x, s.y}, st, (f32x2){b.x, b.y});
    const f32x2 y1 = z2((f32x2){v.z, v.w}, (f32x2){s.z, s.w}, st, (f32x2){b.z, b.w});
    i16x4 o;
    if constexpr (ACT == ACT_GELU || ACT == ACT_QUICKGELU) {
      const f32x2 lo = ACT == ACT_GELU ? gelu_erf2(y0) : quick_gelu2(y0);
      const f32x2 hi = ACT == ACT_GELU ? gelu_erf2(y1) : quick_gelu2(y1);
      o[0] = to_bits<T>(fin(lo[0]));
      o[1] = to_bits<T>(fin(lo[1]));
      o[2] = to_bits<T>(fin(hi[0]));
      o[3] = to_bits<T>(fin(hi[1]));
    } else {
      o[0] = to_bits<T>(y0[0]);
      o[1] = to_bits<T>(y0[1]);
      o[2] = to_bits<T>(y1[0]);
      o[3] = to_bits<T>(y1[1]);
    }
    return o;
  }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4 b) const {
    put4ln<ASM>(r, c, v, b, *(const float4*)(colsum + c), stats[r]);
  }
  MICLIP_DEV void put1(int r, int c, float v, float b) const {
    C[(size_t)r * ldc + c] = to_t<T>(fin(act_fn<ACT>(z(v, colsum[c], stats[r], b))));
  }
};
template <class Epi> struct IsLN : std::false_type {};
template <typename T, int ACT> struct IsLN<EpiStoreLN<T, ACT>> : std::true_type {};
// epilogues with a value form (val4 / val4ln): the persistent GEMM computes their
// tiles with the MFMA operands swapped (a lane then holds 4 consecutive columns of
// one row) and stages the converted outputs
template <class Epi> struct TrAcc : std::false_type {};
template <typename T, int ACT> struct TrAcc<EpiStoreLN<T, ACT>> : std::true_type {};
template <typename T, int ACT> struct TrAcc<EpiStore<T, ACT>> : std::true_type {};

// Residual stream X (R = float, or _Float16 as in the reference's fp16 GPU
// model, clip/model.py:184-185 `x = x + ...` on half tensors) += acc + bias.
// fp16: the reference's two roundings -- the projection's output t = fp16(acc +
// bias), then the half-tensor add x + t, an IEEE fp16 add (v_pk_add_f16; for two
// fp16 operands fp16(float(x) + float(t)) is the same value). Every path (the
// persistent kernel's transposed-accumulator readback, put4x, put1) does exactly
// this, so the tile and tail paths agree bit for bit.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
MICLIP_DEV unsigned add_f16x2(unsigned a, unsigned b) {
  return __builtin_bit_cast(unsigned, __builtin_bit_cast(h16x2, a) + __builtin_bit_cast(h16x2, b));
}
template <typename R>
struct EpiResidual {
  R* X;
  const float* bias;
  int ldx;
  MICLIP_DEV float4 bias4(int col) const { return ld_bias4(bias, col); }
  MICLIP_DEV float4 bias4nb(int col) const { return ld_bias4_nb(bias, col); }
  MICLIP_DEV float bias1(int col) const { return bias[col]; }
  MICLIP_DEV static float fin(float y) {
    asm("" : "+v"(y));
    return y;
  }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4 b) const {
    if constexpr (std::is_same_v<R, float>) {
      float4* p = (float4*)(X + (size_t)r * ldx + c);
      const float4 x = *p;
      const float4 y = make_float4(x.x + (v.x + b.x), x.y + (v.y + b.y), x.z + (v.z + b.z),
                                   x.w + (v.w + b.w));
      if constexpr (ASM)
        st_b128_asm(p, y);
      else
        *p = y;
    } else {
      put4x<ASM>(r, c, v, b, load4(r, c));
    }
  }
  // fp16 stream, split form for the LDS-staged epilogues: a pass's 16 residual
  // rows are loaded (load4) before the accumulators are staged, so their latency
  // hides under the LDS writes instead of sitting in front of every store.
  MICLIP_DEV i16x4 load4(int r, int c) const { return *(const i16x4*)(X + (size_t)r * ldx + c); }
  // fp32 stream (bf16 models): the same split form for the persistent kernel
  MICLIP_DEV f32x4 load4f(int r, int c) const { return *(const f32x4*)(X + (size_t)r * ldx + c); }
  MICLIP_DEV void put4xf(int r, int c, float4 v, float4 b, f32x4 x) const {
    *(f32x4*)(X + (size_t)r * ldx + c) =
        f32x4{x[0] + (v.x + b.x), x[1] + (v.y + b.y), x[2] + (v.z + b.z), x[3] + (v.w + b.w)};
  }
  // fp16 stream: the projection's 4 output elements t = fp16(acc + b), packed
  // adds (v_pk_add_f32) then the conversion -- the value the transposed-
  // accumulator epilogue stages; the residual add follows at readback (add_x)
  MICLIP_DEV i16x4 val4(float4 v, float4 b) const {
    f32x2 y0 = (f32x2){v.x, v.y} + (f32x2){b.x, b.y};
    f32x2 y1 = (f32x2){v.z, v.w} + (f32x2){b.z, b.w};
    asm("" : "+v"(y0), "+v"(y1));
    i16x4 o;
    o[0] = to_bits<R>(y0[0]);
    o[1] = to_bits<R>(y0[1]);
    o[2] = to_bits<R>(y1[0]);
    o[3] = to_bits<R>(y1[1]);
    return o;
  }
  // x + t on n fp16 pairs (dwords)
  template <int NW>
  MICLIP_DEV static void add_x(unsigned (&t)[NW], const unsigned (&x)[NW]) {
#pragma unroll
    for (int i = 0; i < NW; ++i) t[i] = add_f16x2(x[i], t[i]);
  }
  template <bool ASM = false>
  MICLIP_DEV void put4x(int r, int c, float4 v, float4 b, i16x4 x) const {
    const u32x2 t2 = __builtin_bit_cast(u32x2, val4(v, b));
    const u32x2 x2 = __builtin_bit_cast(u32x2, x);
    unsigned t[2] = {t2[0], t2[1]};
    const unsigned xx[2] = {x2[0], x2[1]};
    add_x<2>(t, xx);
    const i16x4 o = __builtin_bit_cast(i16x4, (u32x2){t[0], t[1]});
    i16x4* p = (i16x4*)(X + (size_t)r * ldx + c);
    if constexpr (ASM)
      st_b64_asm(p, o);
    else
      *p = o;
  }
  MICLIP_DEV void put1(int r, int c, float v, float b) const {
    R* p = X + (size_t)r * ldx + c;
    if constexpr (std::is_same_v<R, float>)
      *p = *p + (v + b);
    else
      *p = to_t<R>(fin((float)*p + from_bits<R>(to_bits<R>(fin(v + b)))));
  }
};

// Epilogues whose put4 reads the output first (fp16 residual stream): the
// staged epilogues prefetch those reads (load4 / put4x).
template <class Epi> struct PrefetchX : std::false_type {};
template <> struct PrefetchX<EpiResidual<_Float16>> : std::true_type {};
// the fp16 residual stream runs the transposed-accumulator epilogue too: t is
// staged, and x + t is formed at readback on row-contiguous 16-B pieces
template <> struct TrAcc<EpiResidual<_Float16>> : std::true_type {};
// fp32 residual rows (16 B per lane) are prefetched by the persistent kernel only
// (8 rows per pass; the one-tile kernel's 16 would cost 64 VGPRs)
template <class Epi> struct PrefetchXF : std::false_type {};
template <> struct PrefetchXF<EpiResidual<float>> : std::true_type {};

struct EpiF32 {
  float* C;
  const float* bias;
  int ldc;
  MICLIP_DEV float4 bias4(int col) const { return ld_bias4(bias, col); }
  MICLIP_DEV float4 bias4nb(int col) const { return ld_bias4_nb(bias, col); }
  MICLIP_DEV float bias1(int col) const { return bias ? bias[col] : 0.f; }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4 b) const {
    const float4 y = make_float4(v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
    if constexpr (ASM)
      st_b128_asm(C + (size_t)r * ldc + c, y);
    else
      *(float4*)(C + (size_t)r * ldc + c) = y;
  }
  MICLIP_DEV void put1(int r, int c, float v, float b) const { C[(size_t)r * ldc + c] = v + b; }
};

// Diagnostic: stores only when the (impossible) flag is set, so the MFMA work
// stays live but no output traffic is generated. Used to price the epilogue.
struct EpiNull {
  float* C;
  int flag;
  MICLIP_DEV float4 bias4(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  MICLIP_DEV float4 bias4nb(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  MICLIP_DEV float bias1(int) const { return 0.f; }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4) const {
    if (flag == 12345) *(float4*)(C + c) = v;
  }
  MICLIP_DEV void put1(int r, int c, float v, float) const {
    if (flag == 12345) C[c] = v;
  }
};

template <typename R>
struct EpiPatch {
  R* X;
  const float* pos;
  int ldx;
  int np;
  MICLIP_DEV float4 bias4(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  MICLIP_DEV float4 bias4nb(int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  MICLIP_DEV float bias1(int) const { return 0.f; }
  MICLIP_DEV size_t row_of(int r) const {
    const int b = r / np;
    return (size_t)b * (np + 1) + 1 + (r - b * np);
  }
  template <bool ASM = false>
  MICLIP_DEV void put4(int r, int c, float4 v, float4) const {
    const int p = r % np;
    const float4 q = *(const float4*)(pos + (size_t)(1 + p) * ldx + c);
    const float4 y = make_float4(v.x + q.x, v.y + q.y, v.z + q.z, v.w + q.w);
    if constexpr (std::is_same_v<R, float>) {
      if constexpr (ASM)
        st_b128_asm(X + row_of(r) * ldx + c, y);
      else
        *(float4*)(X + row_of(r) * ldx + c) = y;
    } else {
      i16x4 o;
      o[0] = to_bits<R>(EpiResidual<R>::fin(y.x));
      o[1] = to_bits<R>(EpiResidual<R>::fin(y.y));
      o[2] = to_bits<R>(EpiResidual<R>::fin(y.z));
      o[3] = to_bits<R>(EpiResidual<R>::fin(y.w));
      *(i16x4*)(X + row_of(r) * ldx + c) = o;
    }
  }
  MICLIP_DEV void put1(int r, int c, float v, float) const {
    X[row_of(r) * ldx + c] =
        to_t<R>(EpiResidual<R>::fin(v + pos[(size_t)(1 + r % np) * ldx + c]));
  }
};

}  // namespace

}  // namespace miclip
