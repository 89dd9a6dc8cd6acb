// Fused multi-head attention (head dim 64, or 80 for open_clip ViT-H/14) over
// the packed QKV projection.
//
// Replaces, for one ResidualAttentionBlock, torch's
//   F.multi_head_attention_forward slow path (q.view(tgt_len, bsz*heads, dh) ->
//   scaled_dot_product_attention(q, k, v, attn_mask) -> permute back)
// called from clip/model.py:179-181, with the optional additive causal mask of
// the text tower (clip/model.py:323-329, -inf strictly above the diagonal).
// The N x N score matrix is never materialised (online softmax, fp32).
//
// CDNA4 design:
//   * one workgroup per (image, head); the head's whole K and V (N <= 608 keys,
//     64 dims) are staged once into LDS and shared by all waves;
//   * each wave owns 32-query chunks; S^T = K . Q^T with
//     v_mfma_f32_32x32x16 (swapped operands, cdna_hip_programming.md T12): the
//     query sits on the MFMA lane, so the softmax row max/sum over keys is an
//     in-register reduction plus one lane^32 exchange;
//   * the S^T accumulator is converted in place to the B operand of
//     O^T = V^T . P^T ("accumulator as next operand", §3), and V^T's A
//     fragments come from the row-major V image through ds_read_b64_tr_b16
//     (T10) in the permuted k order that the accumulator layout dictates;
//   * K image XOR-swizzled by (row>>1)&7 (conflict-free ds_read_b128 for the
//     32x32x16 A fragment), V image by (row&3)<<1 (conflict-free tr reads);
//     both layouts were checked with an LDS bank model of gfx950's lane groups.
//   * head dim 80 (HeadGeom<80>): K/V rows padded to 96 dims (192 B; K chunks
//     rotated by (row >> 3) & 3, V unswizzled -- conflict-free at that pitch, see
//     HeadGeom); S^T takes 5 k-steps, O^T three 32-dim tiles of which the last is
//     half padding (zero V columns, never stored).
#include "common.h"
#include "kernels.h"

#include <cmath>
#include <cstdlib>

namespace miclip {

namespace {

constexpr float kLog2e = 1.4426950408889634f;

// Eight ones in fp16 / bf16: the head-dim-80 V image's padding chunk 10 (dims
// 80-87) is DMA'd from here, so the third O^T tile's row 80 accumulates sum_k P
// (the softmax row sum) in the P.V MFMAs themselves (attend_chunk, DH = 80)
__device__ __attribute__((aligned(16))) const unsigned short kOnesF16[8] = {
    0x3C00, 0x3C00, 0x3C00, 0x3C00, 0x3C00, 0x3C00, 0x3C00, 0x3C00};
__device__ __attribute__((aligned(16))) const unsigned short kOnesBF16[8] = {
    0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};

// x (op) x of lane l ^ 32, for every lane: one v_permlane32_swap (gfx950) swaps
// the upper half of one copy with the lower half of the other, so the pair
// {r[0], r[1]} is {x_l, x_(l^32)} in some order. A VALU op; __shfl_xor(x, 32)
// lowers to an LDS ds_bpermute round trip in the middle of every key tile's
// softmax (cdna_hip_programming.md T12).
MICLIP_DEV float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
MICLIP_DEV float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  // same order on both halves (lane l < 32 sees {x_l, x_l+32}, l >= 32 {x_l-32, x_l}):
  // the low half's value first, so both lanes of a pair hold the identical sum
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// LDS geometry of one (image, head)'s K or V image for head dim DH: where logical
// 16-B chunk c of key row `row` sits (kswz / vswz) and which logical chunk a
// physical one holds (kinv / vinv, for the source-side swizzle of the LDS-DMA).
// DH = 64: 128-B rows of 8 chunks; K XOR (row >> 1) & 7, V XOR (row & 3) << 1.
// DH = 80: rows padded to 96 dims (192 B, 12 chunks, a 48-dword pitch): K rotated
// by (row >> 3) & 3 chunks, V unswizzled. Bank model (MI355X_MICROARCH.md LDS
// table): attend_chunk's K ds_read_b128 (rows l32, chunk 2s + hh) and V
// ds_read_b64_tr_b16 (rows 4 (g >> 1) + tq, +8, +16) are then conflict-free --
// 20 / 24 LDS cycles per tile instead of the 40 / 40 of the XOR swizzle the 128-B
// rows use, which is 2-way at this pitch (PMC: SQ_LDS_BANK_CONFLICT 45 % of the
// LDS-active cycles of the head-dim-80 kernel before). V's swizzle must not move
// with row bits 3-4: attend_chunk reads rows +8 / +16 at fixed offsets.
template <int DH>
struct HeadGeom {
  static_assert(DH == 64 || DH == 80, "head dim 64 or 80");
  static constexpr int NKS = DH / 16;         // k-steps of S^T = K . Q^T (32x32x16)
  static constexpr int NDT = (DH + 31) / 32;  // 32-dim tiles of O^T
  static constexpr int ROWB = NDT * 64;       // LDS bytes per key row
  static constexpr int CH = ROWB / 16;        // 16-B chunks per row
  static constexpr int TILEB = 32 * ROWB;     // one 32-key tile
  static MICLIP_DEV int kswz(int c, int row) {
    if constexpr (DH == 64) return c ^ ((row >> 1) & 7);
    const int p = c + ((row >> 3) & 3);
    return p < 12 ? p : p - 12;
  }
  static MICLIP_DEV int kinv(int p, int row) {
    if constexpr (DH == 64) return p ^ ((row >> 1) & 7);
    const int c = p - ((row >> 3) & 3);
    return c >= 0 ? c : c + 12;
  }
  static MICLIP_DEV int vswz(int c, int row) {
    if constexpr (DH == 64) return c ^ ((row & 3) << 1);
    return c;
  }
  static MICLIP_DEV int vinv(int p, int row) { return vswz(p, row); }   // involutions
  // DH = 80: V's padding chunk 10 holds ones, so O^T row 80 is the P row sum
  static constexpr bool ONES = DH == 80;
};

// Head dim 80 with UNPADDED rows (160 B, 10 chunks): the pipelined head-dim-80
// kernel, whose three half-head K/V slots must fit one CU's LDS beside each other
// (3 x 40 KiB). K chunks rotated by row bit 4, V chunks by 2 on even rows: by the
// bank model (MI355X_MICROARCH.md LDS table; the K ds_read_b128 lane groups over
// rows l32, the V ds_read_b64_tr_b16 groups over rows 4 (g >> 1) + tq (+8, +16))
// both are conflict-free -- 20 / 24 LDS cycles per tile. The third O^T tile's dims
// 80-95 do not exist here: its lanes for chunks 10-11 read chunks 8-9 again (same
// address, a broadcast), so O^T rows 80-95 are copies, never stored, and the row
// sum is taken on VALU (ONES = false).
struct HeadGeom80u {
  static constexpr int NKS = 5, NDT = 3, ROWB = 160, CH = 10, TILEB = 32 * ROWB;
  static constexpr bool ONES = false;
  static MICLIP_DEV int kswz(int c, int row) {
    const int p = c + ((row >> 4) & 1);
    return p < 10 ? p : p - 10;
  }
  static MICLIP_DEV int kinv(int p, int row) {
    const int c = p - ((row >> 4) & 1);
    return c >= 0 ? c : c + 10;
  }
  static MICLIP_DEV int vswz(int c, int row) {
    const int p = c + ((row & 1) ? 0 : 2);
    return p < 10 ? p : p - 10;
  }
  static MICLIP_DEV int vinv(int p, int row) {
    const int c = p - ((row & 1) ? 0 : 2);
    return c >= 0 ? c : c + 10;
  }
};

template <typename T>
MICLIP_DEV float dot2acc(uint32_t a, uint32_t b, float c);
template <>
MICLIP_DEV float dot2acc<_Float16>(uint32_t a, uint32_t b, float c) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, a), __builtin_bit_cast(h2, b), c, false);
}
template <>
MICLIP_DEV float dot2acc<__bf16>(uint32_t a, uint32_t b, float c) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, a), __builtin_bit_cast(b2, b), c,
                                         false);
}

// Online softmax of one 32-key score tile S^T (raw scores, masked ones -inf) in
// base 2 with c2 = scale * log2(e) folded into one FMA per element, p =
// exp2(s c2 - m) against the running max m (scaled domain); lazy rescale of lsum
// and O^T (cdna_hip_programming.md T13: the decision precedes the tile's
// exponentials; the old max is kept while the tile max exceeds it by <= 8, p <=
// 2^8, exact range for fp16/bf16 P). Leaves P^T as the P.V MFMA's B operand
// (pf[s2]: accumulator regs 8 s2 .. 8 s2 + 7) and, with SUMP, adds the fp32 row
// sum to lsum. Without (padded head dim 80): the sum rides the P.V MFMAs (V's
// padding dims 80-87 are ones: O^T rows 80-87 = sum_k P).
template <typename T, int NDT, bool SUMP>
MICLIP_DEV void softmax_tile(f32x16& sacc, float c2, float& m, float& lsum, f32x16 (&o)[NDT],
                             i16x8 (&pf)[2]) {
  // a v_max3 tree: 8 ops for 16 values
  const float t0 = fmaxf(fmaxf(sacc[0], sacc[1]), sacc[2]);
  const float t1 = fmaxf(fmaxf(sacc[3], sacc[4]), sacc[5]);
  const float t2 = fmaxf(fmaxf(sacc[6], sacc[7]), sacc[8]);
  const float t3 = fmaxf(fmaxf(sacc[9], sacc[10]), sacc[11]);
  const float t4 = fmaxf(fmaxf(sacc[12], sacc[13]), sacc[14]);
  float tmax = fmaxf(fmaxf(fmaxf(t0, t1), t2), fmaxf(fmaxf(t3, t4), sacc[15]));
  tmax = xor32_max(tmax) * c2;
  if (!__all(tmax - m <= 8.0f)) {
    const float mnew = fmaxf(m, tmax);
    const float alpha = __builtin_amdgcn_exp2f(m - mnew);
    m = mnew;
    lsum *= alpha;
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt][r] *= alpha;
  }
  // raw v_exp_f32: exp2f's denormal-range fix-up (cmp/cndmask/ldexp per
  // element) is dead weight here -- results below 2^-126 vanish in the fp16
  // P operand anyway. Scalar f32 ops on purpose (this file builds with
  // -fno-slp-vectorize): beside MFMAs a v_pk_fma_f32 issues slower than the two
  // scalar ops it replaces (MI355X_MICROARCH.md, per-instruction constants).
  // (four partial sums break the add dependency chain; they start at the first
  // four values: 0 + v == v for the non-negative exponentials)
  float ps[4];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float v = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[r], c2, -m));
    sacc[r] = v;
    if constexpr (SUMP) {
      if (r < 4)
        ps[r] = v;
      else
        ps[r & 3] += v;
    }
  }
  if constexpr (SUMP) lsum += (ps[0] + ps[2]) + (ps[1] + ps[3]);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[s2][j] = to_bits<T>(sacc[8 * s2 + j]);
}

// One wave: 32 queries [32*chunk, +32) of one (image, head) against all keys
// staged in LDS (kimg / vimg). qf: this wave's Q^T fragments (B operand).
// Leaves the unnormalised O^T (o[dt]: d 32*dt .. 32*dt+31) and the row sum
// of this lane's query; attend_store writes the normalised rows.
// kt0 / kt_end: key-tile range (kt_end < 0: all tiles the chunk attends to);
// m: the running max (scaled log2 domain) that lsum and O^T are relative to.
// first / last: a key range processed in several calls starts the online
// softmax state in the first call and reduces lsum across the lane halves in
// the last one (both true: one call over the range).
// G: the K/V image geometry (HeadGeom<DH>, or HeadGeom80u); tile0: the key tile
// held at byte 0 of kimg / vimg (a slot holding tiles tile0.. of the head).
template <typename T, bool CAUSAL, int DH, bool PIPE = true, bool OPQ = false,
          class G = HeadGeom<DH>>
MICLIP_DEV void attend_chunk(const char* kimg, const char* vimg, const i16x8 (&qf)[G::NKS],
                             int chunk, int N, int Npad, float c2, int lane, f32x16 (&o)[G::NDT],
                             float& lsum, float& m, int kt0 = 0, int kt_end = -1, int prio = 0,
                             bool first = true, bool last = true, int tile0 = 0) {
  const int l32 = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int q = chunk * 32 + l32;
  if (first) {
    m = -1e30f;
    lsum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt) o[dt][r] = 0.f;
  }
  const int nkt_all = Npad >> 5;
  const int nkt = kt_end >= 0 ? kt_end
                              : (CAUSAL ? (chunk + 1 < nkt_all ? chunk + 1 : nkt_all) : nkt_all);
  // Per-lane LDS byte offsets inside one 32-key tile (TILEB bytes of K, of V),
  // loop-invariant: the swizzles depend on the key row only through bits that
  // a multiple of 32 rows does not change. Per tile only the two running
  // bases move, so the reads need no per-tile index arithmetic.
  int koff[G::NKS];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s)
    koff[s] = l32 * G::ROWB + (G::kswz(2 * s + hh, l32) << 4);
  int voff[G::NDT];
#pragma unroll
  for (int dt = 0; dt < G::NDT; ++dt) {
    int ch = 4 * dt + 2 * (g & 1) + (tp >> 1);
    if (ch >= G::CH) ch -= 2;   // HeadGeom80u: dims 80-95 re-read 64-79 (never stored)
    voff[dt] = (4 * (g >> 1) + tq) * G::ROWB + (G::vswz(ch, 4 * (g >> 1) + tq) << 4) + 8 * (tp & 1);
  }
  // Two-stage tile pipeline (cdna_hip_programming.md T15): the S^T MFMAs of
  // tile kt+1 are issued before tile kt's softmax, so the matrix pipe works
  // while this wave's VALU runs the exponentials (and the softmax does not
  // wait out the S chain's latency).
  // (prio: every caller passes attn_prio() = 1; the priority raise is unconditional
  // so no per-tile branch on a kernel argument is left in the loop)
  (void)prio;
  // 32-bit LDS addresses (address space 3). OPQ: from an opaque wave-uniform base
  // -- the dynamic-LDS symbol is a relocation hipcc otherwise re-adds to every
  // per-lane offset at every read (6 VALU per key tile); it costs registers, so
  // only the x8 kernel (122 of its 128 VGPRs) takes it (the 16-wave
  // attention_kernel<64> spilled with it)
  unsigned kb = (unsigned)(uintptr_t)(const LDS_AS char*)kimg - tile0 * G::TILEB;
  unsigned vb = (unsigned)(uintptr_t)(const LDS_AS char*)vimg - tile0 * G::TILEB;
  if constexpr (OPQ) asm("" : "+s"(kb), "+s"(vb));
  const LDS_AS char* kl = (const LDS_AS char*)(uintptr_t)kb;
  const LDS_AS char* vl = (const LDS_AS char*)(uintptr_t)vb;
  auto qk = [&](int kt, f32x16& sacc) {
    const LDS_AS char* ktile = kl + kt * G::TILEB;
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      const i16x8 kf = *(const LDS_AS i16x8*)(ktile + koff[s]);
      sacc = Mfma<T>::m32(kf, qf[s], sacc);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto softmax_pv = [&](int kt, f32x16& sacc) {
    const LDS_AS char* vtile = vl + kt * G::TILEB;
    // ---- mask (only tiles that need it), then the online softmax ----
    const bool need_mask = (kt * 32 + 32 > N) || (CAUSAL && kt == chunk);
    if (need_mask) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const bool valid = kk < N && (!CAUSAL || kk <= q);
        sacc[r] = valid ? sacc[r] : -INFINITY;
      }
    }
    i16x8 pf[2];
    softmax_tile<T, G::NDT, !G::ONES>(sacc, c2, m, lsum, o, pf);
    // ---- O^T[d][q] += V^T . P^T ----
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt) {
        // key rows 16*s2 + 4*(g>>1) + tq (+8) of this tile
        const LDS_AS char* a0 = vtile + voff[dt] + 16 * G::ROWB * s2;
        const i16x4 lo = ds_read_tr16_b64(a0);
        const i16x4 hi = ds_read_tr16_b64(a0 + 8 * G::ROWB);  // rows +8 keep (row & 3)
        const i16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[dt] = Mfma<T>::m32(vf, pf[s2], o[dt]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  if constexpr (PIPE) {
    f32x16 sa, sb;
    int kt = kt0;
    if (kt < nkt) qk(kt, sa);
    for (; kt + 2 <= nkt; kt += 2) {
      qk(kt + 1, sb);
      softmax_pv(kt, sa);
      if (kt + 2 < nkt) qk(kt + 2, sa);
      softmax_pv(kt + 1, sb);
    }
    if (kt < nkt) softmax_pv(kt, sa);
  } else {
    // one score tile live (16 fewer VGPRs): for kernels whose latency hiding
    // comes from more waves per SIMD instead of the in-wave pipeline
    f32x16 sa;
    for (int kt = kt0; kt < nkt; ++kt) {
      qk(kt, sa);
      softmax_pv(kt, sa);
    }
  }
  if constexpr (G::ONES) {
    // O^T row 80 (hh = 0 lanes) / 84 (hh = 1): both in the ones chunk, so every
    // lane holds its query's sum of the P values the MFMAs used
    if (last) lsum = o[2][8];
  } else {
    if (last) lsum = xor32_sum(lsum);
  }
}

// Keys [key0, key0 + nkeys) (at most a few: the keys past the last full 32-key
// tile, e.g. key 256 of N = 257) for one wave's 32 queries on VALU instead of a
// 31/32-masked MFMA tile, continuing attend_chunk's online-softmax state (call
// it with last = false and reduce lsum after). Lane (l32, hh) holds dims 16s +
// 8hh + j of query l32 in qf[s][j] and O^T dims 32dt + 8(r>>2) + 4hh + (r&3) in
// o[dt][r]: the score is a half-dot per lane summed across the lane halves
// (v_dot2c_f32: exact fp16 products, fp32 sums), p = exp2(score*c2 - m) with
// the same lazy rescale rule, P rounded to the compute dtype as the MFMA path's
// B operand, and lsum counts p once (lane half 0). DH = 64 images (x8 kernel).
template <typename T>
MICLIP_DEV void attend_extra_keys(const char* kimg, const char* vimg, const i16x8 (&qf)[4],
                                  f32x16 (&o)[2], float& lsum, float& m, int key0, int nkeys,
                                  float c2, int lane, int row0 = 0) {
  // row0: key row held at byte 0 of kimg / vimg (a streamed key-tile slot);
  // the swizzles still follow the absolute key row k
  const int hh = lane >> 5;
  for (int k = key0; k < key0 + nkeys; ++k) {
    const char* kr = kimg + (k - row0) * 128;
    float part = 0.f;
    // (memory clobbers keep the LDS reads from being hoisted together: the
    // x8 kernel runs at its 128-VGPR cap)
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const u32x4 kv = *(const u32x4*)(kr + (((2 * st + hh) ^ ((k >> 1) & 7)) << 4));
      const u32x4 qv = __builtin_bit_cast(u32x4, qf[st]);
#pragma unroll
      for (int e = 0; e < 4; ++e) part = dot2acc<T>(qv[e], kv[e], part);
      asm volatile("" ::: "memory");
    }
    const float score = xor32_sum(part);
    const float sc = score * c2;
    if (!__all(sc - m <= 8.0f)) {
      const float mnew = fmaxf(m, sc);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      m = mnew;
      lsum *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o[0][r] *= alpha;
        o[1][r] *= alpha;
      }
    }
    const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(score, c2, -m));
    if (hh == 0) lsum += p;
    const float p16 = to_f<T>(to_t<T>(p));
    const char* vr = vimg + (k - row0) * 128;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        const int ch = 4 * dt + rq;   // 16-B chunk of dims 32dt + 8rq .. +7
        const i16x4 v = *(const i16x4*)(vr + ((ch ^ ((k & 3) << 1)) << 4) + 8 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[dt][4 * rq + e] = __builtin_fmaf(p16, from_bits<T>(v[e]), o[dt][4 * rq + e]);
        asm volatile("" ::: "memory");
      }
  }
}

// Full key tiles [kt0, kt1) of one wave's 32 queries with the softmax's per-element
// VALU work moved onto the matrix pipe (the x8, one-head N = 577 and head-dim-80
// kernels; they were VALU-bound: r04 PMC 22 % MFMA busy at 17 VALU per MFMA, the
// tile loop issuing ~75 VALU + 16 v_exp per 8 MFMAs):
//  * Q arrives pre-scaled by c2 = scale * log2(e) (prescale_q: one fp32 product and
//    one rounding per element, once per chunk), so S' = K . Q'^T is already in the
//    base-2 softmax domain;
//  * the running max leaves through the MFMA chain: every tile's S' chain starts
//    with a shift k-step ones . (-m~)^T (A = 1 in k-slot 0 of the first lane half,
//    B = -m~ rounded to the compute dtype there, zeros elsewhere), so the
//    accumulator holds S' - m~ and p = exp2(acc) takes no per-element FMA (m~ only
//    has to be one shift per row: p, l and O all use it);
//  * the lazy-rescale test is one v_max3 tree against the threshold per lane (the
//    wave vote covers both lane halves; no lane exchange on the fast path);
//  * the row sum is a v_dot2 of the rounded P pairs with ones -- the sum of exactly
//    the P values the P.V MFMAs use -- 8 ops instead of 16 adds;
//  * NT > 0: the NT tiles are unrolled, every LDS read a per-lane base + immediate.
// PIPE: tile kt+1's S MFMAs are issued before tile kt's softmax (a max update in
// tile kt then corrects the in-flight tile by the same shift). `fresh`: the first
// call of a chunk (o, l zeroed; m~ set from the first tile's max). Leaves the
// unnormalised O^T, this lane's partial row sum (reduce across the lane halves
// after any further keys) and m~ (scaled log2 domain: attend_extra_keys with c2 = 1).
// tile0: the key tile held at byte 0 of kimg / vimg. All tiles must be full (no
// masking: kt1 * 32 <= N, not causal).
template <typename T, class G>
MICLIP_DEV void prescale_q(i16x8 (&qf)[G::NKS], float c2) {
#pragma unroll
  for (int s = 0; s < G::NKS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[s][j] = to_bits<T>(from_bits<T>(qf[s][j]) * c2);
}

template <typename T, class G, bool PIPE, int NT = 0>
MICLIP_DEV void attend_shift(const char* kimg, const char* vimg, const i16x8 (&qf)[G::NKS],
                             int lane, f32x16 (&o)[G::NDT], float& lsum, float& m, int kt0,
                             int kt1, bool fresh, int tile0 = 0) {
  const int l32 = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  unsigned kb = (unsigned)(uintptr_t)(const LDS_AS char*)kimg;
  unsigned vb = (unsigned)(uintptr_t)(const LDS_AS char*)vimg;
  asm("" : "+s"(kb), "+s"(vb));
  const LDS_AS char* kp[G::NKS];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s)
    kp[s] = (const LDS_AS char*)(uintptr_t)(kb + l32 * G::ROWB + (G::kswz(2 * s + hh, l32) << 4));
  const LDS_AS char* vp[G::NDT];
#pragma unroll
  for (int dt = 0; dt < G::NDT; ++dt) {
    int ch = 4 * dt + 2 * (g & 1) + (tp >> 1);
    if (ch >= G::CH) ch -= 2;   // HeadGeom80u: dims 80-95 re-read 64-79 (never stored)
    const int vr = 4 * (g >> 1) + tq;
    vp[dt] = (const LDS_AS char*)(uintptr_t)(vb + vr * G::ROWB + (G::vswz(ch, vr) << 4) + 8 * (tp & 1));
  }
  const short one = to_bits<T>(1.0f);
  const i16x8 ka = {hh == 0 ? one : (short)0, 0, 0, 0, 0, 0, 0, 0};
  i16x8 qm = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t ones2 = (uint32_t)(unsigned short)one * 0x10001u;
  if (fresh) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt) o[dt][r] = 0.f;
    lsum = 0.f;
    m = 0.f;
  } else {
    qm[0] = hh == 0 ? to_bits<T>(-m) : (short)0;
  }
  auto qk = [&](int kt, f32x16& sacc) {
    const int off = (kt - tile0) * G::TILEB;
    __builtin_amdgcn_s_setprio(1);
    const i16x8 k0 = *(const LDS_AS i16x8*)(kp[0] + off);
    sacc = Mfma<T>::m32(ka, qm, f32x16{});
    sacc = Mfma<T>::m32(k0, qf[0], sacc);
#pragma unroll
    for (int s = 1; s < G::NKS; ++s) {
      const i16x8 kf = *(const LDS_AS i16x8*)(kp[s] + off);
      sacc = Mfma<T>::m32(kf, qf[s], sacc);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // nxt: the tile in flight behind this one (PIPE), corrected by a max update when
  // has_nxt (a reference, never a pointer: a pointer to one of two register tiles
  // picked at run time put both in scratch)
  auto softmax_pv = [&](int kt, f32x16& sacc, f32x16& nxt, bool has_nxt) {
    const float t0 = fmaxf(fmaxf(sacc[0], sacc[1]), sacc[2]);
    const float t1 = fmaxf(fmaxf(sacc[3], sacc[4]), sacc[5]);
    const float t2 = fmaxf(fmaxf(sacc[6], sacc[7]), sacc[8]);
    const float t3 = fmaxf(fmaxf(sacc[9], sacc[10]), sacc[11]);
    const float t4 = fmaxf(fmaxf(sacc[12], sacc[13]), sacc[14]);
    const float tmax = fmaxf(fmaxf(fmaxf(t0, t1), t2), fmaxf(fmaxf(t3, t4), sacc[15]));
    if (fresh || !__all(tmax <= 8.0f)) {
      // first tile of the chunk, or a tile max more than 2^8 above m~: m~ = the row
      // max (both lane halves), rounded to the compute dtype; O and l rescaled
      const float rmax = xor32_max(tmax) + m;   // absolute, scaled log2 domain
      const float mn = from_bits<T>(to_bits<T>(fresh ? rmax : fmaxf(m, rmax)));
      const float d = mn - m;
      if (!fresh) {
        const float alpha = __builtin_amdgcn_exp2f(-d);
        lsum *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
          for (int dt = 0; dt < G::NDT; ++dt) o[dt][r] *= alpha;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] -= d;
      if (has_nxt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) nxt[r] -= d;
      }
      m = mn;
      qm[0] = hh == 0 ? to_bits<T>(-mn) : (short)0;
      fresh = false;
    }
    i16x8 pf[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = __builtin_amdgcn_exp2f(sacc[r]);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[s2][j] = to_bits<T>(sacc[8 * s2 + j]);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const u32x4 w = __builtin_bit_cast(u32x4, pf[s2]);
#pragma unroll
      for (int e = 0; e < 4; ++e) lsum = dot2acc<T>(w[e], ones2, lsum);
    }
    const int off = (kt - tile0) * G::TILEB;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt) {
        const LDS_AS char* a0 = vp[dt] + off + 16 * G::ROWB * s2;
        const i16x4 lo = ds_read_tr16_b64(a0);
        const i16x4 hi = ds_read_tr16_b64(a0 + 8 * G::ROWB);
        const i16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[dt] = Mfma<T>::m32(vf, pf[s2], o[dt]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  if constexpr (NT > 0) {
    if constexpr (PIPE) {
      f32x16 sa, sb;
      qk(kt0, sa);
#pragma unroll
      for (int i = 0; i < NT; i += 2) {
        if (i + 1 < NT) qk(kt0 + i + 1, sb);
        softmax_pv(kt0 + i, sa, sb, i + 1 < NT);
        if (i + 1 < NT) {
          if (i + 2 < NT) qk(kt0 + i + 2, sa);
          softmax_pv(kt0 + i + 1, sb, sa, i + 2 < NT);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        f32x16 sa;
        qk(kt0 + i, sa);
        softmax_pv(kt0 + i, sa, sa, false);
      }
    }
  } else if constexpr (PIPE) {
    f32x16 sa, sb;
    int kt = kt0;
    if (kt < kt1) qk(kt, sa);
    for (; kt + 2 <= kt1; kt += 2) {
      qk(kt + 1, sb);
      softmax_pv(kt, sa, sb, true);
      const bool more = kt + 2 < kt1;
      if (more) qk(kt + 2, sa);
      softmax_pv(kt + 1, sb, sa, more);
    }
    if (kt < kt1) softmax_pv(kt, sa, sb, false);
  } else {
    for (int kt = kt0; kt < kt1; ++kt) {
      f32x16 sa;
      qk(kt, sa);
      softmax_pv(kt, sa, sa, false);
    }
  }
}

template <typename T, int DH>
MICLIP_DEV void attend_store(const f32x16 (&o)[HeadGeom<DH>::NDT], float lsum, int chunk, int N,
                             T* op_row0, int D, int lane) {
  const int hh = lane >> 5;
  const int q = chunk * 32 + (lane & 31);
  const float inv = 1.0f / lsum;
  // Lane (l32, hh) holds dims 8rg + 4hh .. +3 of query l32 for rg = 0..3 of each
  // 32-dim tile. Per rg pair one v_permlane32_swap per dword (guide T21) leaves
  // lane hh = 0 with dims 8rg .. 8rg+7 and lane hh = 1 with dims 8rg+8 .. 8rg+15:
  // 16-B stores, half the store instructions. The swaps run on the full wave;
  // the pair of lanes exchanging shares its query, hence the row guard.
  T* op = op_row0 + (size_t)(q < N ? q : 0) * D;
#pragma unroll
  for (int dt = 0; dt < HeadGeom<DH>::NDT; ++dt) {
#pragma unroll
    for (int rg = 0; rg < 4; rg += 2) {
      if (32 * dt + 8 * rg >= DH) continue;  // padding dims (DH = 80: rg 2-3 of tile 2)
      i16x4 w0, w1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w0[e] = to_bits<T>(o[dt][4 * rg + e] * inv);
        w1[e] = to_bits<T>(o[dt][4 * rg + 4 + e] * inv);
      }
      const u32x2 a = __builtin_bit_cast(u32x2, w0), b = __builtin_bit_cast(u32x2, w1);
      const auto s0 = __builtin_amdgcn_permlane32_swap(a[0], b[0], false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(a[1], b[1], false, false);
      const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
      if (q < N) *(u32x4*)(op + 32 * dt + 8 * rg + 8 * hh) = v;
    }
  }
}

// Padding queries (q >= N) load row N-1: a query only ever meets its own
// S^T column, P^T column and O^T column, and padding rows are never stored,
// so finite duplicate data is as good as zeros -- and the load stays
// branch-free (a zeroing else-branch makes hipcc wait vmcnt(0) for the
// registers' previous loads at every head, draining the K/V DMA).
template <typename T, int DH>
MICLIP_DEV void load_q(i16x8 (&qf)[HeadGeom<DH>::NKS], const T* base, int ld, int chunk, int N,
                       int lane) {
  int q = chunk * 32 + (lane & 31);
  q = q < N ? q : N - 1;
  const T* qp = base + (size_t)q * ld + 8 * (lane >> 5);
#pragma unroll
  for (int s = 0; s < HeadGeom<DH>::NKS; ++s) qf[s] = *(const i16x8*)(qp + 16 * s);
}

// One workgroup per (image, head). Launch bounds: NWMAX waves -- DH = 64: 12
// (3 per SIMD, 132 VGPRs) or 16 (4 per SIMD, 128 VGPRs, one spill outside the key
// loop), see attn_launch_plain; DH = 80 carries a third O^T tile and a fifth Q
// fragment and just fits the 168 VGPRs of 9 waves (3 on one SIMD): one wave
// per 32-query chunk at N = 257 (8 waves left one wave two chunks).
template <typename T, bool CAUSAL, int DH, int NWMAX = (DH == 64 ? 12 : 9)>
__global__ __launch_bounds__(NWMAX * 64) void attention_kernel(
    const T* __restrict__ qkv, T* __restrict__ out, int N, int H, int Npad, int nchunks,
    float qk_scale, int prio) {
  using G = HeadGeom<DH>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  char* kimg = smem;                  // [Npad][ROWB/2] T
  char* vimg = smem + Npad * G::ROWB;  // [Npad][ROWB/2] T

  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const T* base = qkv + (size_t)b * N * ld + h * DH;

  if constexpr (DH == 64) {
    // K / V images by LDS-DMA, 1-KiB pieces of 8 rows, the swizzle applied to
    // the SOURCE chunk (as the x8 kernel stages them): every piece is issued
    // before any wait. (The register path below loaded 2 x 16 B per thread and
    // waited for them before its next pair -- ~8 serial round trips per head
    // at N = 577.) Pad rows repeat row N - 1: finite data under masked keys.
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const int prow = lane >> 3, pch = lane & 7, pieces = Npad / 8;
    for (int pc = wave; pc < 2 * pieces; pc += nwv) {
      const bool isv = pc >= pieces;
      const int piece = isv ? pc - pieces : pc;
      const int row = piece * 8 + prow;
      const int r = row < N ? row : N - 1;
      const int lch = isv ? (pch ^ ((row & 3) << 1)) : (pch ^ ((row >> 1) & 7));
      glds16_hidden(base + (size_t)r * ld + (isv ? 2 * D : D) + lch * 8,
                    (isv ? vimg : kimg) + piece * 1024);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    // head dim 80: the same all-DMAs-then-one-wait staging over 192-B rows. A
    // 1-KiB piece covers 5 1/3 rows, so each lane finds the (row, physical chunk)
    // its 16 bytes land on and fetches the logical chunk there (HeadGeom::kinv /
    // vinv, the inverse swizzles). Padding chunks (dims 80-95) take dims
    // 16-31 of the same row -- finite; K's are never read (5 k-steps cover dims
    // 0-79), V's only feed O^T rows 80-95, which are never stored. Pad rows repeat
    // row N - 1. (The register path this replaces loaded 2 x 16 B per thread and
    // waited before each LDS write: 6 serial round trips per head at N = 257.)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const int pieces = Npad * G::ROWB / 1024;   // Npad % 32 == 0: whole pieces
    for (int pc = wave; pc < 2 * pieces; pc += nwv) {
      const bool isv = pc >= pieces;
      const int piece = isv ? pc - pieces : pc;
      const int off = piece * 1024 + lane * 16;
      const int row = off / G::ROWB, pch = (off - row * G::ROWB) >> 4;
      int c = isv ? G::vinv(pch, row) : G::kinv(pch, row);
      const T* src;
      if (isv && c == DH / 8) {   // V dims 80-87: ones (the row sum, see kOnesF16)
        src = (const T*)(std::is_same_v<T, _Float16> ? kOnesF16 : kOnesBF16);
      } else {
        if (c * 8 >= DH) c -= 8;
        const int r = row < N ? row : N - 1;
        src = base + (size_t)r * ld + (isv ? 2 * D : D) + c * 8;
      }
      glds16_hidden(src, (isv ? vimg : kimg) + piece * 1024);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const float c2 = qk_scale * kLog2e;
  // A last key tile holding 1-3 keys (N = 32k + 1..3, e.g. ViT-L/14@336's 577) is
  // not run as a 29/32-to-31/32-masked MFMA tile: its keys go through
  // attend_extra_keys on VALU (as the x8 kernel's key 256), 1/19 of the key loop
  // at N = 577. Same staging swizzles (DH = 64).
  const int nfull = N >> 5, nextra = N - 32 * nfull;
  const bool xkeys = DH == 64 && !CAUSAL && nextra > 0 && nextra <= 3 && nfull >= 2;
  for (int chunk = wave; chunk < nchunks; chunk += nw) {
    i16x8 qf[G::NKS];
    load_q<T, DH>(qf, base, ld, chunk, N, lane);
    f32x16 o[G::NDT];
    float lsum, m;
    if constexpr (DH == 64 && !CAUSAL) {
      if (xkeys) {
        // Q in the base-2 softmax domain (attend_shift); the extra keys take c2 = 1
        prescale_q<T, G>(qf, c2);
        attend_shift<T, G, true>(kimg, vimg, qf, lane, o, lsum, m, 0, nfull, true);
        attend_extra_keys<T>(kimg, vimg, qf, o, lsum, m, 32 * nfull, nextra, 1.0f, lane);
        lsum = xor32_sum(lsum);
        attend_store<T, DH>(o, lsum, chunk, N, out + (size_t)b * N * D + h * DH, D, lane);
        continue;
      }
    }
    attend_chunk<T, CAUSAL, DH>(kimg, vimg, qf, chunk, N, Npad, c2, lane, o, lsum, m, 0, -1,
                                prio);
    attend_store<T, DH>(o, lsum, chunk, N, out + (size_t)b * N * D + h * DH, D, lane);
  }
}

MICLIP_DEV void wait_vm_upto(int n) {   // s_waitcnt vmcnt(n), n a small run-time count
  switch (n) {
#define MICLIP_VMU(k) \
  case k:           \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MICLIP_VMU(1) MICLIP_VMU(2) MICLIP_VMU(3) MICLIP_VMU(4) MICLIP_VMU(5) MICLIP_VMU(6)
    MICLIP_VMU(7) MICLIP_VMU(8) MICLIP_VMU(9) MICLIP_VMU(10) MICLIP_VMU(11) MICLIP_VMU(12)
#undef MICLIP_VMU
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Head dim 80 (open_clip ViT-H/14, C5), default. attention_kernel<80> holds 110 KiB
// of K/V, so it runs one workgroup per CU and waits for a head's whole fetch before
// any MFMA. Here Q goes to LDS by DMA too (an unpadded 160-B-row image, 45 KiB at
// N = 257; its ds_read_b128 Q fragments are conflict-free at that pitch) and the
// fetch runs in two phases: Q + key tiles 0-3 of K and V, then the rest. Each wave
// waits only for its own phase-A pieces (vmcnt = its phase-B count), the workgroup
// syncs, and every wave runs its query chunk over key tiles 0-3 while phase B lands;
// then a full wait + barrier and tiles 4.. (attend_chunk continuing the online
// softmax). Same data (padding rows repeat row N - 1), same per-tile arithmetic in
// the same order as attention_kernel: bit-identical. One chunk per wave.
template <typename T>
__global__ __launch_bounds__(576) void attention80s_kernel(const T* __restrict__ qkv,
                                                           T* __restrict__ out, int N, int H,
                                                           int Npad, int nchunks, float qk_scale,
                                                           int prio) {
  using G = HeadGeom<80>;
  constexpr int QROWB = 160;   // Q image row: dims 0-79
  constexpr int TA = 4;        // key tiles in phase A
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  char* kimg = smem;
  char* vimg = smem + Npad * G::ROWB;
  char* qimg = smem + 2 * Npad * G::ROWB;
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - b * H;
  const int D = H * 80, ld = 3 * D;
  const T* base = qkv + (size_t)b * N * ld + h * 80;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int kvp = Npad * G::ROWB / 1024;   // 1-KiB pieces per K (or V) image
  const int kva = TA * G::TILEB / 1024;    // ... of which phase A
  const int qp = Npad * QROWB / 1024;      // Q pieces (Npad % 32 == 0: whole pieces)
  // attention_kernel<80>'s K / V staging of one piece (192-B rows, swizzled chunks)
  auto kv_piece = [&](bool isv, int piece) {
    const int off = piece * 1024 + lane * 16;
    const int row = off / G::ROWB, pch = (off - row * G::ROWB) >> 4;
    int c = isv ? G::vinv(pch, row) : G::kinv(pch, row);
    const T* src;
    if (isv && c == 80 / 8) {
      src = (const T*)(std::is_same_v<T, _Float16> ? kOnesF16 : kOnesBF16);
    } else {
      if (c * 8 >= 80) c -= 8;
      const int r = row < N ? row : N - 1;
      src = base + (size_t)r * ld + (isv ? 2 * D : D) + c * 8;
    }
    glds16_hidden(src, (isv ? vimg : kimg) + piece * 1024);
  };
  auto q_piece = [&](int piece) {   // padding queries: row N - 1, as load_q
    const int off = piece * 1024 + lane * 16;
    const int row = off / QROWB, ch = (off - row * QROWB) >> 4;
    const int r = row < N ? row : N - 1;
    glds16_hidden(base + (size_t)r * ld + ch * 8, qimg + piece * 1024);
  };
  const int nA = qp + 2 * kva, nB = 2 * (kvp - kva), half = kvp - kva;
  for (int pc = wave; pc < nA; pc += nw) {
    if (pc < qp) {
      q_piece(pc);
    } else {
      const int i = pc - qp;
      kv_piece(i >= kva, i >= kva ? i - kva : i);
    }
  }
  for (int pc = wave; pc < nB; pc += nw) kv_piece(pc >= half, kva + (pc >= half ? pc - half : pc));
  wait_vm_upto(wave < nB ? (nB - wave + nw - 1) / nw : 0);   // this wave's phase A landed
  __syncthreads();

  const float c2 = qk_scale * kLog2e;
  const int chunk = wave;
  f32x16 o[G::NDT];
  float lsum = 0.f, m = 0.f;
  i16x8 qf[G::NKS];
  const int l32 = lane & 31, hh = lane >> 5;
  if (chunk < nchunks) {
    const char* qrow = qimg + (chunk * 32 + l32) * QROWB + hh * 16;
#pragma unroll
    for (int s2 = 0; s2 < G::NKS; ++s2) qf[s2] = *(const i16x8*)(qrow + 32 * s2);
    attend_chunk<T, false, 80>(kimg, vimg, qf, chunk, N, Npad, c2, lane, o, lsum, m, 0, TA, prio,
                               true, false);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (chunk < nchunks) {
    attend_chunk<T, false, 80>(kimg, vimg, qf, chunk, N, Npad, c2, lane, o, lsum, m, TA, -1, prio,
                               false, true);
    attend_store<T, 80>(o, lsum, chunk, N, out + (size_t)b * N * D + h * 80, D, lane);
  }
}

// Keys [0, nkeys) of the unpadded 160-B-row images kx / vx (the keys past the 8
// full tiles, at most 3) for one wave's 32 queries on VALU, continuing
// attend_chunk's online-softmax state: attend_extra_keys (head dim 64) over the
// five 16-dim Q fragments and the three O^T tiles (dims 80-95 of the third are
// copies, left alone). Call attend_chunk with last = false and reduce lsum after.
template <typename T>
MICLIP_DEV void attend_extra_keys80u(const char* kx, const char* vx, const i16x8 (&qf)[5],
                                     f32x16 (&o)[3], float& lsum, float& m, int nkeys, float c2,
                                     int lane) {
  const int hh = lane >> 5;
  for (int k = 0; k < nkeys; ++k) {
    const char* kr = kx + k * 160;
    float part = 0.f;
#pragma unroll
    for (int st = 0; st < 5; ++st) {
      const u32x4 kv = *(const u32x4*)(kr + ((2 * st + hh) << 4));
      const u32x4 qv = __builtin_bit_cast(u32x4, qf[st]);
#pragma unroll
      for (int e = 0; e < 4; ++e) part = dot2acc<T>(qv[e], kv[e], part);
      asm volatile("" ::: "memory");
    }
    const float score = xor32_sum(part);
    const float sc = score * c2;
    if (!__all(sc - m <= 8.0f)) {
      const float mnew = fmaxf(m, sc);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      m = mnew;
      lsum *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o[0][r] *= alpha;
        o[1][r] *= alpha;
        o[2][r] *= alpha;
      }
    }
    const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(score, c2, -m));
    if (hh == 0) lsum += p;
    const float p16 = to_f<T>(to_t<T>(p));
    const char* vr = vx + k * 160;
#pragma unroll
    for (int dt = 0; dt < 3; ++dt)
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        if (dt == 2 && rq >= 2) continue;   // dims 80-95: none
        const i16x4 v = *(const i16x4*)(vr + ((4 * dt + rq) << 4) + 8 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[dt][4 * rq + e] = __builtin_fmaf(p16, from_bits<T>(v[e]), o[dt][4 * rq + e]);
        asm volatile("" ::: "memory");
      }
  }
}

// Head dim 80, pipelined (default at N = 256..259: open_clip ViT-H/14 at 224 px,
// C5). attention80s_kernel holds a whole head (110 KiB) and so runs one head at a
// time per CU, fetch then compute: 2.25 waves per SIMD, 9 query chunks over 4
// SIMDs (one SIMD carries 3), the 257th key as a 31/32-masked ninth tile. Here one
// workgroup (8 waves, 2 per SIMD: the register budget is 256) walks hpw heads with
// the K/V images in half-head units (key tiles 0-3, 4-7; 40 KiB of unpadded
// 160-B rows, HeadGeom80u) in a ring of three slots: while a wave computes unit u,
// units u + 1 and u + 2 are in flight, so a head's fetch runs under the previous
// head's MFMAs. Wave w owns query chunk w over the 8 full key tiles, then the keys
// past them (N - 256 <= 3, staged beside the slots) on VALU; the ragged query chunk
// (N - 256 queries) is dealt flash-decoding style, key tile w to wave w (waves 0-3
// in the first half, 4-7 in the second: one of each per SIMD), wave 7 also its
// extra keys, and wave c merges query c's 8 partials (LDS, fixed order) after the
// head's closing barrier. Q fragments of the next head load into registers during
// the second half; hipcc's wait for them at the head boundary also retires the
// (older) DMAs of the next head. Online-softmax arithmetic per tile as
// attend_chunk's; the row sum is taken on VALU (no ones chunk in 160-B rows).
template <typename T>
__global__ __launch_bounds__(512) void attention80p_kernel(const T* __restrict__ qkv,
                                                           T* __restrict__ out, int B, int N,
                                                           int H, int hpw, float qk_scale,
                                                           int prio) {
  using G = HeadGeom80u;
  constexpr int HALFB = 128 * G::ROWB;   // 20 KiB: key tiles 0-3 (or 4-7) of K or V
  constexpr int SLOTB = 2 * HALFB;       // one unit: K half, then V half
  constexpr int PSTR = 84;               // partial: 80 dims, m, lsum (+2)
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  char* ximg = smem + 3 * SLOTB;                       // [2 parity][K | V | Q, 1 KiB each]
  float* part = (float*)(smem + 3 * SLOTB + 6144);     // [2 parity][8 waves][3][PSTR]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nvalid = N - 256;   // ragged queries = keys past the 8 full tiles (0..3)
  const int D = H * 80, ld = 3 * D;
  const float c2 = qk_scale * kLog2e;
  const int bh0 = blockIdx.x * hpw;
  const int nh = (B * H - bh0) < hpw ? (B * H - bh0) : hpw;
  if (nh <= 0) return;   // workgroup-uniform
  auto head_base = [&](int bh) {
    const int b = bh / H, h = bh - b * H;
    return qkv + (size_t)b * N * ld + h * 80;
  };
  // unit (head at base, half): K and V rows 128 half .. +127 into `slot`, 40
  // 1-KiB pieces (5 per wave), the swizzle applied to the source chunk
  // opaque lane index: per-lane offsets are recomputed at each use instead of
  // hoisted out of the head loop for every inlined call site (which spilled)
  auto olane = [&]() {
    int l = lane;
    asm volatile("" : "+v"(l));
    return l;
  };
  auto stage_half = [&](const T* base, int half, int slot) {
    char* img = smem + slot * SLOTB;
    const int lane = olane();
    const u32x4s desc = make_buffer_desc(base);   // 32-bit offsets from the head's row 0
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int pc = wave + 8 * i;
      const bool isv = pc >= 20;
      const int piece = isv ? pc - 20 : pc;
      const int off = piece * 1024 + lane * 16;
      const int rl = off / G::ROWB, pch = (off - rl * G::ROWB) >> 4;
      const int row = 128 * half + rl;
      const int c = isv ? G::vinv(pch, row) : G::kinv(pch, row);
      blds16_hidden(desc, (unsigned)(row * ld + (isv ? 2 * D : D) + c * 8) * (unsigned)sizeof(T),
                    img + (isv ? HALFB : 0) + piece * 1024);
    }
  };
  // rows 256.. (clamped to N - 1; unswizzled 160-B rows) of K (wave 0), V (wave
  // 1) and Q (wave 2): the keys past the 8 full tiles and the ragged queries
  auto stage_extra = [&](const T* base, int par) {
    if (wave < 3) {
      const int lane = olane();
      const int off = lane * 16, rl = off / G::ROWB, ch = (off - rl * G::ROWB) >> 4;
      const int r = 256 + rl < N ? 256 + rl : N - 1;
      glds16_hidden(base + (size_t)r * ld + (wave == 0 ? D : wave == 1 ? 2 * D : 0) + ch * 8,
                    ximg + par * 3072 + wave * 1024);
    }
  };
  // the ragged chunk's Q fragments (load_q's layout) from the staged rows: query
  // lanes past the valid ones read row 0 (finite, never stored)
  auto ragged_q = [&](i16x8 (&qx)[5], int par) {
    const int lane = olane();
    const int l32 = lane & 31, hh = lane >> 5;
    const char* qrow = ximg + par * 3072 + 2048 + (l32 < nvalid ? l32 : 0) * G::ROWB + hh * 16;
#pragma unroll
    for (int s = 0; s < 5; ++s) qx[s] = *(const i16x8*)(qrow + 32 * s);
  };
  // this wave's partial of the ragged queries: lane (l32, hh) holds O^T rows d =
  // (r & 3) + 8 (r >> 2) + 4 hh (+32 dt) of query l32
  auto put_part = [&](const f32x16 (&ox)[3], float mx, float lx, int par) {
    const int l32 = lane & 31, hh = lane >> 5;
    if (l32 < nvalid) {
      float* pw = part + ((par * 8 + wave) * 3 + l32) * PSTR;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = (r & 3) + 8 * (r >> 2) + 4 * hh;
        pw[d] = ox[0][r];
        pw[32 + d] = ox[1][r];
        if (r < 8) pw[64 + d] = ox[2][r];
      }
      if (hh == 0) {
        pw[80] = mx;
        pw[81] = lx;
      }
    }
  };
  // wave c < nvalid: ragged query c of head bh from its 8 partials, in wave order;
  // lane = output dim (lanes 0-15 also dims 64-79)
  auto merge = [&](int bh, int par) {
    if (wave < nvalid) {
      const int b = bh / H, h = bh - b * H;
      const float* pc = part + (par * 8 * 3 + wave) * PSTR;
      float mx = -1e30f;
#pragma unroll
      for (int i = 0; i < 8; ++i) mx = fmaxf(mx, pc[i * 3 * PSTR + 80]);
      float l = 0.f, a0 = 0.f, a1 = 0.f;
      const int d1 = 64 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float* pi = pc + i * 3 * PSTR;
        const float w = __builtin_amdgcn_exp2f(pi[80] - mx);
        l += w * pi[81];
        a0 += w * pi[lane];
        a1 += w * pi[d1];
      }
      T* orow = out + ((size_t)b * N + 256 + wave) * D + h * 80;
      orow[lane] = to_t<T>(a0 / l);
      if (lane < 16) orow[64 + lane] = to_t<T>(a1 / l);
    }
  };

  i16x8 qf[5], qn[5];
  {
    const T* base = head_base(bh0);
    stage_half(base, 0, 0);
    stage_half(base, 1, 1);
    if (nvalid > 0) stage_extra(base, 0);
    load_q<T, 80>(qf, base, ld, wave, N, lane);
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]), "+v"(qf[4])
                 :
                 : "memory");
    prescale_q<T, G>(qf, c2);   // the full chunk runs in the base-2 domain (attend_shift)
  }
  __builtin_amdgcn_s_barrier();
  for (int j = 0; j < nh; ++j) {
    const int bh = bh0 + j, b = bh / H, h = bh - b * H;
    const int sa = (2 * j) % 3, sb = (2 * j + 1) % 3, sn = (2 * j + 2) % 3;
    const bool more = j + 1 < nh;
    const T* nbase = head_base(more ? bh + 1 : bh);
    // ---- first half: key tiles 0-3 in slot sa. Unit (j+1, 0) -> slot sn, the
    // slot of unit (j-1, 1), which every wave left before the barrier above ----
    if (more) stage_half(nbase, 0, sn);
    if (j > 0) merge(bh - 1, (j - 1) & 1);
    const char* ia = smem + sa * SLOTB;
    // (the ragged tile first and the chunk's stores before the second half's
    // ragged tile: the two O^T sets are never live together)
    if (nvalid > 0 && wave < 4) {
      f32x16 ox[3];
      float lx, mx;
      i16x8 qx[5];
      ragged_q(qx, j & 1);
      attend_chunk<T, false, 80, true, false, G>(ia, ia + HALFB, qx, 8, N, 256, c2, olane(), ox, lx,
                                                 mx, wave, wave + 1, prio, true, true, 0);
      put_part(ox, mx, lx, j & 1);
    }
    f32x16 o[3];
    float lsum, m;
    attend_shift<T, G, true, 4>(ia, ia + HALFB, qf, olane(), o, lsum, m, 0, 4, true, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- second half: key tiles 4-7 in slot sb. Unit (j+1, 1) -> slot sa (just
    // left), the next head's extra keys (the other parity) and Q fragments ----
    if (more) {
      stage_half(nbase, 1, sa);
      if (nvalid > 0) stage_extra(nbase, (j + 1) & 1);
      load_q<T, 80>(qn, nbase, ld, wave, N, lane);
    }
    const char* ib = smem + sb * SLOTB;
    const char* ix = ximg + (j & 1) * 3072;
    attend_shift<T, G, true, 4>(ib, ib + HALFB, qf, olane(), o, lsum, m, 4, 8, false, 4);
    if (nvalid > 0) attend_extra_keys80u<T>(ix, ix + 1024, qf, o, lsum, m, nvalid, 1.0f, olane());
    lsum = xor32_sum(lsum);
    if (more) {
      // hipcc waits for these loads here (vmcnt(0): nothing younger is visible to
      // it -- the output stores come after), which also retires the next head's
      // older DMAs before the barrier
#pragma unroll
      for (int s = 0; s < 5; ++s) qf[s] = qn[s];
      asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]), "+v"(qf[4]));
      prescale_q<T, G>(qf, c2);
    }
    attend_store<T, 80>(o, lsum, wave, N, out + (size_t)b * N * D + h * 80, D, lane);
    if (nvalid > 0 && wave >= 4) {
      f32x16 ox[3];
      float lx, mx;
      i16x8 qx[5];
      ragged_q(qx, j & 1);
      attend_chunk<T, false, 80, true, false, G>(ib, ib + HALFB, qx, 8, N, 256, c2, olane(), ox, lx,
                                                 mx, wave, wave + 1, prio, true, false, 4);
      if (wave == 7) attend_extra_keys80u<T>(ix, ix + 1024, qx, ox, lx, mx, nvalid, c2, olane());
      lx = xor32_sum(lx);
      put_part(ox, mx, lx, j & 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  merge(bh0 + nh - 1, (nh - 1) & 1);
}


// ---------------------------------------------------------------------------
// Pipelined form: one workgroup walks hpw consecutive (image, head) pairs.
// While head j is computed, head j+1's K and V are LDS-DMA'd
// (global_load_lds_dwordx4 issued from inline asm, 1-KiB pieces of 8 rows,
// the K/V swizzles applied to the SOURCE address) into the other LDS buffer
// and each wave's Q fragments for head j+1 are loaded into registers, so the
// K/V/Q fetch of the next head runs under this head's MFMA + softmax work.
// One barrier per head: at its top every wave has retired its own DMA and Q
// loads and finished reading the buffer that the next DMA overwrites.
//
// Waves: one per full 32-query chunk. When the last chunk holds only 1-2
// valid queries (`split`; N = 257 = 8*32 + 1: the CLS token row), a ninth
// wave doing a whole chunk's work would put 3 waves on one SIMD and 2 on the
// others. Instead each of the 8 waves, after its own chunk, also takes a
// contiguous range of that chunk's key tiles (nchunks tiles over nw waves),
// leaves a partial (o, m, l) per valid query in LDS, and wave 0 merges the
// partials after the next barrier (flash-decoding style; the same softmax
// arithmetic up to the fp32 order of the merge).
// ---------------------------------------------------------------------------
template <typename T, bool CAUSAL, bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 512 : 640) void attention_pipe_kernel(
    const T* __restrict__ qkv, T* __restrict__ out, int B, int N, int H, int Npad, int hpw,
    float qk_scale, int prio) {
  constexpr bool split = SPLIT;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int img_bytes = Npad * 128;            // one K or V image
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;              // nchunks, or nchunks - 1 when split
  const int nchunks = Npad >> 5;
  const int last = nchunks - 1;                // the split chunk
  const int nvalid = N - 32 * last;            // its valid queries
  // this wave's key-tile range of the split chunk
  const int xkt0 = wave * nchunks / nw, xkt1 = (wave + 1) * nchunks / nw;
  float* part = (float*)(smem + 4 * img_bytes);   // [2][nw][nvalid][66]
  const int D = H * 64, ld = 3 * D;
  const float c2 = qk_scale * kLog2e;
  const int bh0 = blockIdx.x * hpw;
  const int nh = (B * H - bh0) < hpw ? (B * H - bh0) : hpw;
  const int pieces = Npad / 8;                 // 1-KiB pieces per image
  const int prow = lane >> 3, pch = lane & 7;

  auto head_base = [&](int bh) {
    const int b = bh / H, h = bh - b * H;
    return qkv + (size_t)b * N * ld + h * 64;
  };
  auto stage = [&](int bh, int buf) {
    const T* base = head_base(bh);
    char* kimg = smem + buf * 2 * img_bytes;
    char* vimg = kimg + img_bytes;
    for (int pc = wave; pc < 2 * pieces; pc += nw) {
      const bool isv = pc >= pieces;
      const int piece = isv ? pc - pieces : pc;
      const int row = piece * 8 + prow;
      const int r = row < N ? row : N - 1;       // pad rows: finite data, masked keys
      const int lch = isv ? (pch ^ ((row & 3) << 1)) : (pch ^ ((row >> 1) & 7));
      glds16_hidden(base + (size_t)r * ld + (isv ? 2 * D : D) + lch * 8,
                    (isv ? vimg : kimg) + piece * 1024);
    }
  };
  // wave 0: merge head bh's partials (LDS parity par) into its output rows
  auto merge = [&](int bh, int par) {
    const int b = bh / H, h = bh - b * H;
    for (int c = 0; c < nvalid; ++c) {
      const float* pc = part + ((size_t)(par * nw) * nvalid + c) * 66;
      float mx = -1e30f;
      for (int i = 0; i < nw; ++i) mx = fmaxf(mx, pc[(size_t)i * nvalid * 66 + 64]);
      float l = 0.f, o = 0.f;
      for (int i = 0; i < nw; ++i) {
        const float* pi = pc + (size_t)i * nvalid * 66;
        const float w = __builtin_amdgcn_exp2f(pi[64] - mx);
        l += w * pi[65];
        o += w * pi[lane];
      }
      out[((size_t)b * N + 32 * last + c) * D + h * 64 + lane] = to_t<T>(o / l);
    }
  };

  i16x8 qf[4], qn[4], qx[4], qxn[4];
  stage(bh0, 0);
  load_q<T, 64>(qf, head_base(bh0), ld, wave, N, lane);
  if (split) load_q<T, 64>(qx, head_base(bh0), ld, last, N, lane);
  // retire head 0's DMA and Q loads; qf / qx named as outputs so hipcc sees
  // them defined here (guide §5.7 item 1)
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]), "+v"(qx[0]), "+v"(qx[1]),
                 "+v"(qx[2]), "+v"(qx[3])
               :
               : "memory");
  for (int j = 0; j < nh; ++j) {
    const int bh = bh0 + j, b = bh / H, h = bh - b * H;
    // every wave retired its DMA of head j (prologue, or the q <- qn copies of
    // head j-1, below) and its partial writes before this barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (j + 1 < nh) {
      stage(bh + 1, (j + 1) & 1);
      load_q<T, 64>(qn, head_base(bh + 1), ld, wave, N, lane);
      if (split) load_q<T, 64>(qxn, head_base(bh + 1), ld, last, N, lane);
    }
    if (split && wave == 0 && j > 0) merge(bh - 1, (j - 1) & 1);
    const char* kimg = smem + (j & 1) * 2 * img_bytes;
    f32x16 o[2];
    float lsum, m;
    attend_chunk<T, CAUSAL, 64>(kimg, kimg + img_bytes, qf, wave, N, Npad, c2, lane, o, lsum, m,
                                0, -1, prio);
    // Take head j+1's Q BEFORE this head's output stores: hipcc's wait for
    // the qn loads (which also retires the older DMA of head j+1) then never
    // waits for the stores, which drain under the next head's work.
    if (j + 1 < nh) {
#pragma unroll
      for (int s = 0; s < 4; ++s) qf[s] = qn[s];
      asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]));
    }
    attend_store<T, 64>(o, lsum, wave, N, out + (size_t)b * N * D + h * 64, D, lane);
    if (split) {
      attend_chunk<T, CAUSAL, 64>(kimg, kimg + img_bytes, qx, last, N, Npad, c2, lane, o, lsum, m,
                                  xkt0, xkt1);
      if (j + 1 < nh) {
#pragma unroll
        for (int s = 0; s < 4; ++s) qx[s] = qxn[s];
        asm volatile("" : "+v"(qx[0]), "+v"(qx[1]), "+v"(qx[2]), "+v"(qx[3]));
      }
      // partial for the valid queries: lane (l32, hh) holds O^T rows
      // d = (r&3) + 8*(r>>2) + 4*hh (+32 in o1) of query column l32
      const int l32 = lane & 31, hh = lane >> 5;
      if (l32 < nvalid) {
        float* pw = part + ((size_t)((j & 1) * nw + wave) * nvalid + l32) * 66;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = (r & 3) + 8 * (r >> 2) + 4 * hh;
          pw[d] = o[0][r];
          pw[32 + d] = o[1][r];
        }
        if (hh == 0) {
          pw[64] = m;
          pw[65] = lsum;
        }
      }
    }
  }
  if (split) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wave == 0 && nh > 0) merge(bh0 + nh - 1, (nh - 1) & 1);
  }
}

// ---------------------------------------------------------------------------
// Two workgroups per CU (variant 8, default for 8 full query chunks and at most
// 3 more queries, N in 256..259: ViT-L/14 at 224 px). One workgroup = 8 waves (2 per
// SIMD) walks hpw (image, head) pairs with ONE K/V buffer (Npad x 256 B, 72 KiB
// at N = 257), so two workgroups share a CU: while one stages its next head's
// K/V (LDS-DMA) the other computes, and 4 waves per SIMD hide the softmax /
// LDS latencies that 2-3 waves of one workgroup leave exposed (the register
// budget is 128 VGPRs: __launch_bounds__(512, 4)). Wave w owns query chunk w
// (8 x 32 queries) over the 8 full key tiles plus the N - 256 keys past them
// on VALU (attend_extra_keys: no 31/32-masked ninth tile) and, flash-decoding
// style, key tile w of the ragged last chunk (N - 256 queries: the 257th
// token; wave 7 also its extra keys); its partial (m, l, o) per valid query
// goes to LDS; wave v computes the extra keys' partial of ragged query v before
// the head's closing barrier and merges the nine partials after it, in a fixed
// order.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(512, 4) void attention_x8_kernel(const T* __restrict__ qkv,
                                                             T* __restrict__ out, int B, int N,
                                                             int H, int Npad, int hpw,
                                                             float qk_scale, int prio) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int img_bytes = Npad * 128;
  char* kimg = smem;
  char* vimg = smem + img_bytes;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = Npad >> 5;              // key tiles (= query chunks incl. the ragged one)
  const int nvalid = N - 256;                // queries of the ragged chunk 8 (0 = none)
  const int nextra = N - 256;                // keys past the 8 full tiles (attend_extra_keys)
  (void)ntiles;
  float* part = (float*)(smem + 2 * img_bytes);   // [8 waves][nvalid][66]
  const int D = H * 64, ld = 3 * D;
  const float c2 = qk_scale * kLog2e;
  const int bh0 = blockIdx.x * hpw;
  const int nh = (B * H - bh0) < hpw ? (B * H - bh0) : hpw;
  // 1-KiB pieces (8 key rows) per image: only rows < N are ever read (the full
  // tiles cover 0..255, keys past them go through attend_extra_keys / the merge)
  const int pieces = (N + 7) / 8;
  const int prow = lane >> 3, pch = lane & 7;
  auto head_base = [&](int bh) {
    const int b = bh / H, h = bh - b * H;
    return qkv + (size_t)b * N * ld + h * 64;
  };
  MICLIP_STAMP_BEGIN;
  for (int j = 0; j < nh; ++j) {
    const int bh = bh0 + j, b = bh / H, h = bh - b * H;
    const T* base = head_base(bh);
    // every wave finished reading the previous head's K/V (the closing barrier
    // below: the extra keys are taken before it) before these DMAs overwrite them.
    // buffer_load ... lds from a per-head resource: 32-bit offsets (rows clamped, so
    // always inside the image) instead of a 64-bit address product per piece
    for (int pc = wave; pc < 2 * pieces; pc += 8) {
      const bool isv = pc >= pieces;
      const int piece = isv ? pc - pieces : pc;
      const int row = piece * 8 + prow;
      const int r = row < N ? row : N - 1;   // pad rows: finite data, masked keys
      const int lch = isv ? (pch ^ ((row & 3) << 1)) : (pch ^ ((row >> 1) & 7));
      glds16_hidden(base + (unsigned)(r * ld + (isv ? 2 * D : D) + lch * 8),
                    (isv ? vimg : kimg) + piece * 1024);
    }
    MICLIP_STAMP(6);   // DMA issue
    i16x8 qf[4];
    load_q<T, 64>(qf, base, ld, wave, N, lane);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3])::"memory");
    MICLIP_STAMP(7);   // Q loads + wait for everything
    __builtin_amdgcn_s_barrier();
    MICLIP_STAMP(0);   // the barrier
    T* obase = out + (size_t)b * N * D + h * 64;
    {
      f32x16 o[2];
      float lsum, m;
      // Q in the base-2 softmax domain: the full chunk and its extra keys take c2 = 1
      prescale_q<T, HeadGeom<64>>(qf, c2);
      attend_shift<T, HeadGeom<64>, false, 8>(kimg, vimg, qf, lane, o, lsum, m, 0, 8, true);
      attend_extra_keys<T>(kimg, vimg, qf, o, lsum, m, 256, nextra, 1.0f, lane);
      lsum = xor32_sum(lsum);
      MICLIP_STAMP(1);   // the wave's full query chunk
      attend_store<T, 64>(o, lsum, wave, N, obase, D, lane);
      MICLIP_STAMP(2);   // its output stores
    }
    if (nvalid > 0) {
      load_q<T, 64>(qf, base, ld, 8, N, lane);
      f32x16 o[2];
      float lsum, m;
      // key tile `wave` of the 8 full ones (the keys past them: in the merge)
      attend_chunk<T, false, 64, false, true>(kimg, vimg, qf, 8, N, Npad, c2, lane, o, lsum, m,
                                              wave, wave + 1, prio);
      // lane (l32, hh) holds O^T rows d = (r&3) + 8*(r>>2) + 4*hh (+32 in o[1]) of query l32
      const int l32 = lane & 31, hh = lane >> 5;
      if (l32 < nvalid) {
        float* pw = part + ((size_t)wave * nvalid + l32) * 66;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = (r & 3) + 8 * (r >> 2) + 4 * hh;
          pw[d] = o[0][r];
          pw[32 + d] = o[1][r];
        }
        if (hh == 0) {
          pw[64] = m;
          pw[65] = lsum;
        }
      }
    }
    // The keys past the 8 full tiles join the ragged chunk's query c as a ninth
    // partial, computed by wave c BEFORE the closing barrier (lane = dim: the dot
    // product by a wave sum) while this head's K / V rows are still resident:
    // after that barrier the other waves start the next head's DMA into the same
    // image, so nothing below the barrier may read kimg / vimg. nvalid <= 3 < 8,
    // so a wave holds at most one query.
    float me = -1e30f, le = 0.f, oe = 0.f;
    if (wave < nvalid) {
      const float qd = to_f<T>(base[(size_t)(256 + wave) * ld + lane]);
      const int ch = lane >> 3;
      for (int k = 256; k < N; ++k) {
        const float kd = to_f<T>(*(const T*)(kimg + k * 128 + ((ch ^ ((k >> 1) & 7)) << 4) + (lane & 7) * 2));
        const float sc = wave_sum(qd * kd) * c2;
        const float mn = fmaxf(me, sc), al = __builtin_amdgcn_exp2f(me - mn);
        const float p = __builtin_amdgcn_exp2f(sc - mn);
        const float vd = to_f<T>(*(const T*)(vimg + k * 128 + ((ch ^ ((k & 3) << 1)) << 4) + (lane & 7) * 2));
        le = le * al + p;
        oe = oe * al + to_f<T>(to_t<T>(p)) * vd;
        me = mn;
      }
    }
    MICLIP_STAMP(3);     // ragged chunk's key-tile slice + partial + extra keys
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    MICLIP_STAMP(4);     // closing barrier
    // merge the ragged chunk: wave c takes query c; lane = output dim. Reads only
    // the partials, which the next head's partial writes cannot reach before its
    // first barrier (every merging wave joins it after the merge).
    if (wave < nvalid) {
      const float* pc = part + (size_t)wave * 66;
      float mx = me;
#pragma unroll
      for (int i = 0; i < 8; ++i) mx = fmaxf(mx, pc[(size_t)i * nvalid * 66 + 64]);
      const float we = __builtin_amdgcn_exp2f(me - mx);
      float l = we * le, acc = we * oe;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float* pi = pc + (size_t)i * nvalid * 66;
        const float w = __builtin_amdgcn_exp2f(pi[64] - mx);
        l += w * pi[65];
        acc += w * pi[lane];
      }
      obase[(size_t)(256 + wave) * D + lane] = to_t<T>(acc / l);
    }
    MICLIP_STAMP(5);     // merge
  }
  MICLIP_STAMP_END(blockIdx.x * 8 + wave);
}


// ---------------------------------------------------------------------------
// One query per (image, head): token row 0 (CLS) only. The vision tower's last
// block feeds nothing but the CLS rows forward (VisionTransformer.forward,
// clip/model.py:226-229: ln_post(x[:, 0, :])), so there the attention of the
// other N-1 queries is dead work. One workgroup (4 waves) per (image, head),
// on VALU (1 x N x dh MACs per head; K / V rows stream from the QKV buffer):
// thread t scores keys t, t+256, .. with v_dot2c_f32_{f16,bf16} (fp32 sums of
// the exact fp16 products), exponentials in base 2 relative to the row max,
// P rounded to the compute dtype for P.V as in the MFMA kernels (whose B
// operand it is there); P.V by (key group, output dim pair) threads in fp32,
// the key groups summed in a fixed order. out: compact [B, H*dh] (row b =
// image b's CLS row).
// ---------------------------------------------------------------------------
constexpr int kQ0MaxN = 768;   // keys per head (3 per thread)

template <typename T, int DH>
__global__ __launch_bounds__(256) void attention_q0_kernel(const T* __restrict__ qkv,
                                                           T* __restrict__ out, int B, int N,
                                                           int H, float c2) {
  constexpr int NV = DH / 8;          // 16-B vectors per row
  constexpr int NP = DH / 2;          // output dim pairs
  constexpr int KG = 256 / NP;        // key groups of the P.V step (8 for dh 64, 6 for 80)
  constexpr int NJ = kQ0MaxN / 256;   // key passes
  __shared__ float sp[kQ0MaxN];       // p per key
  __shared__ float red[KG][DH];       // per key group partial P.V; [0][0..7]: reductions
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const T* base = qkv + (size_t)b * N * ld + h * DH;
  u32x4 qv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) qv[i] = *(const u32x4*)(base + 8 * i);
  float sc[NJ];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int k = t + 256 * j;
    float a = -INFINITY;
    if (256 * j < N) {                // block-uniform pass guard
      const T* kr = base + (size_t)(k < N ? k : N - 1) * ld + D;
      u32x4 kv[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) kv[i] = *(const u32x4*)(kr + 8 * i);
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = dot2acc<T>(qv[i][e], kv[i][e], acc);
      a = k < N ? acc * c2 : -INFINITY;
    }
    sc[j] = a;
    mx = fmaxf(mx, a);
  }
  float* rw = &red[0][0];
  mx = wave_max(mx);
  if (lane == 0) rw[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(rw[0], rw[1]), fmaxf(rw[2], rw[3]));
  float ls = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float pj = __builtin_amdgcn_exp2f(sc[j] - mx);   // exp2(-inf) = 0 past N
    ls += pj;
    if (t + 256 * j < kQ0MaxN) sp[t + 256 * j] = pj;
  }
  ls = wave_sum(ls);
  __syncthreads();                    // everyone read rw[0..3] (max) before reuse
  if (lane == 0) rw[4 + wave] = ls;
  // P.V: thread (g, dp), g < KG: keys k = g, g + KG, ..; output dims 2dp, 2dp+1
  const int g = t / NP, dp = t - g * NP;
  float a0 = 0.f, a1 = 0.f;
  if (g < KG) {
    const T* vb = base + 2 * D + 2 * dp;
    for (int k = g; k < N; k += KG) {
      const uint32_t v = *(const uint32_t*)(vb + (size_t)k * ld);
      const float p16 = to_f<T>(to_t<T>(sp[k]));
      a0 = __builtin_fmaf(p16, from_bits<T>((short)(v & 0xffff)), a0);
      a1 = __builtin_fmaf(p16, from_bits<T>((short)(v >> 16)), a1);
    }
  }
  __syncthreads();                    // rw[4..7] visible; sp reads done
  const float lsum = (rw[4] + rw[5]) + (rw[6] + rw[7]);
  __syncthreads();                    // before red[] is overwritten below
  if (g < KG) {
    red[g][2 * dp] = a0;
    red[g][2 * dp + 1] = a1;
  }
  __syncthreads();
  if (t < DH) {
    float o = 0.f;
#pragma unroll
    for (int q = 0; q < KG; ++q) o += red[q][t];
    out[(size_t)b * D + h * DH + t] = to_t<T>(o / lsum);
  }
}

// Attention kernel variants are chosen by the op-level `variant` argument only
// (miclip_op_attention, A/B benches); the model path always runs variant 0.
// s_setprio 1 around each tile's MFMA issue: with 2-3 waves per SIMD the one
// issuing MFMAs goes first, the others' softmax VALU fills its gaps (ViT-L/14
// layer: 0.184 -> 0.177 ms, same-box A/B).
constexpr int attn_prio() { return 1; }

// one workgroup per (image, head)
template <typename T, bool CAUSAL, int DH>
hipError_t attn_launch_plain(const void* qkv, void* out, int B, int N, int H, hipStream_t s,
                             int waves = 0) {
  using G = HeadGeom<DH>;
  const int Npad = (N + 31) & ~31;
  const int nchunks = Npad / 32;
  const size_t lds = (size_t)Npad * G::ROWB * 2;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // Waves: DH 80 at most 9 (the fewest that keep the chunks per wave). DH 64: one
  // per chunk up to 16 (4 per SIMD, attention_kernel<.., 16>). A wave's chunks run
  // serially and a SIMD's waves share its issue, so the count sets both the longest
  // chain and the per-SIMD load: at N = 577 (18 full chunks + one 1-query chunk)
  // 10 waves put 6 chunks on one SIMD (waves 0, 4, 8), 12 or 16 waves at most 5 --
  // 0.312-0.322 (10) -> 0.287-0.303 (12) / 0.284-0.296 ms (16) per B = 128 launch,
  // bit-identical (scripts/probe/attn_waves.py, profiles/r04/configs/attn577_waves.jsonl).
  // `waves` (variants 10-16) forces a count for that probe. With the extra keys on
  // VALU (N = 32k + 1..3, non-causal) the 16-wave build spills (6 VGPRs at its 128 cap)
  // and 12 waves win: N = 577, B = 256: 0.569-0.575 (12) vs 0.592-0.595 ms (16),
  // 0.590-0.596 before the change (profiles/r05/attn577/ab.txt).
  int nw;
  if constexpr (DH == 64) {
    const int xk = N & 31;
    const int cap = (!CAUSAL && xk >= 1 && xk <= 3 && N >= 64) ? 12 : 16;
    nw = nchunks < cap ? nchunks : cap;
    if (waves > 0) {
      if (waves > 16) return hipErrorInvalidValue;
      nw = waves < nchunks ? waves : nchunks;
    }
  } else {
    if (waves > 0) return hipErrorInvalidValue;
    const int per = (nchunks + 8) / 9;
    nw = (nchunks + per - 1) / per;
  }
  void (*kern)(const T*, T*, int, int, int, int, float, int);
  if constexpr (DH == 64)
    kern = nw > 12 ? attention_kernel<T, CAUSAL, DH, 16> : attention_kernel<T, CAUSAL, DH, 12>;
  else
    kern = attention_kernel<T, CAUSAL, DH>;
  static bool attr_set[2] = {false, false};
  if (!attr_set[nw > 12]) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set[nw > 12] = true;
  }
  hipLaunchKernelGGL(kern, dim3(B * H), dim3(nw * 64), lds, s, (const T*)qkv, (T*)out, N, H,
                     Npad, nchunks, 1.0f / sqrtf((float)DH), attn_prio());
  return hipGetLastError();
}

template <typename T, bool CAUSAL>
hipError_t attn_launch(const void* qkv, void* out, int B, int N, int H, int dh, hipStream_t s,
                       int variant) {
  if (dh == 80) {
    // the pipelined kernel (default; variant 6) at 8 full query chunks + at most 3
    // more queries; else the two-phase kernel (variant 2) where a chunk per wave fits
    // 9 waves and Q's image fits beside K / V; variant 1 = attention_kernel<80>
    if (variant == 6 || (variant == 0 && !CAUSAL && N >= 256 && N <= 259)) {
      if (CAUSAL || N < 256 || N > 259) return hipErrorInvalidValue;
      constexpr size_t lds80p = 3 * 2 * 128 * 160 + 6144 + 2 * 8 * 3 * 84 * 4;
      static bool a80p = false;
      if (!a80p) {
        const hipError_t e = hipFuncSetAttribute((const void*)attention80p_kernel<T>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lds80p);
        if (e != hipSuccess) return e;
        a80p = true;
      }
      static int ncu80 = [] {
        int d = 0, n = 0;
        if (hipGetDevice(&d) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
          n = 256;
        return n;
      }();
      const int heads = B * H;
      int hpw = (heads + ncu80 - 1) / ncu80;
      hpw = hpw < 1 ? 1 : hpw;
      const int grid = (heads + hpw - 1) / hpw;
      hipLaunchKernelGGL((attention80p_kernel<T>), dim3(grid), dim3(512), lds80p, s, (const T*)qkv,
                         (T*)out, B, N, H, hpw, 1.0f / sqrtf(80.f), attn_prio());
      return hipGetLastError();
    }
    const int Npad = (N + 31) & ~31, nchunks = Npad / 32;
    const size_t lds80 = (size_t)Npad * (2 * HeadGeom<80>::ROWB + 160);
    if (!CAUSAL && variant != 1 && nchunks <= 9 && Npad >= 160 && lds80 <= 160 * 1024) {
      static bool a80 = false;
      if (!a80) {
        const hipError_t e = hipFuncSetAttribute((const void*)attention80s_kernel<T>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024);
        if (e != hipSuccess) return e;
        a80 = true;
      }
      hipLaunchKernelGGL((attention80s_kernel<T>), dim3(B * H), dim3(nchunks * 64), lds80, s,
                         (const T*)qkv, (T*)out, N, H, Npad, nchunks, 1.0f / sqrtf(80.f),
                         attn_prio());
      return hipGetLastError();
    }
    if (variant == 2) return hipErrorInvalidValue;   // the two-phase kernel does not apply
    return attn_launch_plain<T, CAUSAL, 80>(qkv, out, B, N, H, s);
  }
  if (dh != 64) return hipErrorInvalidValue;
  const int Npad = (N + 31) & ~31;
  const int nchunks = Npad / 32;
  const size_t lds = (size_t)Npad * 256;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // two workgroups per CU (default when the queries are 8 full chunks + a small
  // ragged one: K/V (72 KiB) plus the partials of 8 waves x the ragged queries
  // must stay under 80 KiB of LDS, i.e. N - 256 <= 3)
  const size_t lds_x8 = lds + (size_t)8 * (N > 256 ? N - 256 : 0) * 66 * 4;
  if (variant == 9) return hipErrorInvalidValue;   // removed (measured level)
  if (variant == 8 || (!CAUSAL && variant == 0 && N >= 256 && N < 288 && lds_x8 <= 80 * 1024)) {
    // at most 3 ragged queries: one per merging wave (attention_x8_kernel)
    if (CAUSAL || N < 256 || N > 259 || lds_x8 > 80 * 1024) return hipErrorInvalidValue;
    static bool x8_attr = false;
    if (!x8_attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)attention_x8_kernel<T>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               80 * 1024);
      if (e != hipSuccess) return e;
      x8_attr = true;
    }
    static int ncu8 = [] {
      int d = 0, n = 0;
      if (hipGetDevice(&d) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
        n = 256;
      return n;
    }();
    const int heads = B * H, slots = 2 * ncu8;
    int hpw = (heads + slots - 1) / slots;
    hpw = hpw < 1 ? 1 : hpw;
    const int grid = (heads + hpw - 1) / hpw;
    hipLaunchKernelGGL((attention_x8_kernel<T>), dim3(grid), dim3(512), lds_x8, s, (const T*)qkv,
                       (T*)out, B, N, H, Npad, hpw, 0.125f, attn_prio());
    return hipGetLastError();
  }
  // pipelined kernel (default; variant 2): two K/V buffers must fit in LDS
  // (N <= 320). ViT-L/14 layer: 0.19-0.21 ms vs 0.21-0.24 ms one head per WG.
  if (variant != 1 && variant != 3 && variant < 10 && 2 * lds + 2 * 10 * 2 * 66 * 4 <= 160 * 1024) {
    static bool attr_set = false;
    if (!attr_set) {
      for (const void* k : {(const void*)attention_pipe_kernel<T, CAUSAL, false>,
                            (const void*)attention_pipe_kernel<T, CAUSAL, true>}) {
        const hipError_t e =
            hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
      }
      attr_set = true;
    }
    // one round of workgroups over the CUs at the occupancy LDS allows
    static int ncu = [] {
      int d = 0, n = 0;
      if (hipGetDevice(&d) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
        n = 256;
      return n;
    }();
    // split the last chunk's key tiles over the other waves when it holds 1-2 queries
    const int nvalid = N - 32 * (nchunks - 1);
    const bool split = !CAUSAL && nchunks >= 5 && nvalid <= 2 && variant == 4;
    const int waves = split ? nchunks - 1 : nchunks;
    const size_t lds_all = 2 * lds + (split ? (size_t)2 * waves * nvalid * 66 * 4 : 0);
    const int per_cu = (int)((160 * 1024) / lds_all) < 1 ? 1 : (int)((160 * 1024) / lds_all);
    const int heads = B * H, slots = ncu * per_cu;
    int hpw = (heads + slots - 1) / slots;
    hpw = hpw < 1 ? 1 : hpw;
    const int grid = (heads + hpw - 1) / hpw;
    if (split)
      hipLaunchKernelGGL((attention_pipe_kernel<T, CAUSAL, true>), dim3(grid), dim3(waves * 64),
                         lds_all, s, (const T*)qkv, (T*)out, B, N, H, Npad, hpw, 0.125f,
                         attn_prio());
    else
      hipLaunchKernelGGL((attention_pipe_kernel<T, CAUSAL, false>), dim3(grid), dim3(waves * 64),
                         lds_all, s, (const T*)qkv, (T*)out, B, N, H, Npad, hpw, 0.125f,
                         attn_prio());
    return hipGetLastError();
  }
  if (variant == 3) return hipErrorInvalidValue;
  return attn_launch_plain<T, CAUSAL, 64>(qkv, out, B, N, H, s, variant >= 10 ? variant : 0);
}

}  // namespace

hipError_t attention_q0(int dtype, const void* qkv, void* out, int B, int N, int H,
                        hipStream_t s, int head_dim) {
  if (B < 1 || N < 1 || H < 1 || N > kQ0MaxN) return hipErrorInvalidValue;
  if (head_dim == 0) head_dim = 64;
  if (head_dim != 64 && head_dim != 80) return hipErrorInvalidValue;
  const int grid = B * H;
  const float c2 = kLog2e / sqrtf((float)head_dim);
  if (dtype == kF16) {
    if (head_dim == 64)
      hipLaunchKernelGGL((attention_q0_kernel<_Float16, 64>), dim3(grid), dim3(256), 0, s,
                         (const _Float16*)qkv, (_Float16*)out, B, N, H, c2);
    else
      hipLaunchKernelGGL((attention_q0_kernel<_Float16, 80>), dim3(grid), dim3(256), 0, s,
                         (const _Float16*)qkv, (_Float16*)out, B, N, H, c2);
  } else {
    if (head_dim == 64)
      hipLaunchKernelGGL((attention_q0_kernel<__bf16, 64>), dim3(grid), dim3(256), 0, s,
                         (const __bf16*)qkv, (__bf16*)out, B, N, H, c2);
    else
      hipLaunchKernelGGL((attention_q0_kernel<__bf16, 80>), dim3(grid), dim3(256), 0, s,
                         (const __bf16*)qkv, (__bf16*)out, B, N, H, c2);
  }
  return hipGetLastError();
}

hipError_t attention(int dtype, const void* qkv, void* out, int B, int N, int H, int causal,
                     hipStream_t s, int variant, int head_dim) {
  if (B < 1 || N < 1 || H < 1) return hipErrorInvalidValue;
  if (dtype == kF16)
    return causal ? attn_launch<_Float16, true>(qkv, out, B, N, H, head_dim, s, variant)
                  : attn_launch<_Float16, false>(qkv, out, B, N, H, head_dim, s, variant);
  return causal ? attn_launch<__bf16, true>(qkv, out, B, N, H, head_dim, s, variant)
                : attn_launch<__bf16, false>(qkv, out, B, N, H, head_dim, s, variant);
}

}  // namespace miclip
