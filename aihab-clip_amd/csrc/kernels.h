// Host-side launchers of the miclip CDNA4 kernels (internal interface).
// Every launcher validates the shapes its kernel assumes and returns
// hipErrorInvalidValue instead of launching when they do not hold.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "miclip.h"

namespace miclip {

// ACT_GELU_TANH: GELU's tanh form, used only where the result is quantised to
// MX-fp8 next (gemm_mx epi 5): its <= 4.8e-4 deviation from the exact GELU is far
// below the e4m3 step (2^-3 relative)
enum Act { ACT_NONE = 0, ACT_QUICKGELU = 1, ACT_GELU = 2, ACT_GELU_TANH = 3 };

// ---- GEMM: C[M,N] = A[M,K] . W[N,K]^T (+ epilogue); A, W in compute dtype ----
// Shapes: N % 128 == 0, K % 64 == 0, any M >= 1; A, W rows K-contiguous.
// Store epilogue: C (compute dtype, ld = N) = act(acc + bias).
// `variant`: 0 = pick by size, 128 / 256 = force that tile (tests, A/B timing).
// skws / sk (the GEMMs of the CLS-only last block): split K into sk deterministic
// slices through an fp32 workspace skws of sk * M * N floats (K % (64 sk) == 0)
hipError_t gemm_store(int dtype, const void* A, const void* W, const float* bias, void* C,
                      int M, int N, int K, int act, hipStream_t s, int variant = 0,
                      float* skws = nullptr, int sk = 1);
// LayerNorm folded into the GEMM (epilogue.h, EpiStoreLN): A = the un-normalised
// rows, W = W diag(gamma) (ln_fold), stats [M] float2 {mean, rstd} (ln_stats);
// C = act(rstd * (acc - mean * colsum) + c).
hipError_t gemm_store_ln(int dtype, const void* A, const void* W, const float* c,
                         const float* colsum, const void* stats, void* C, int M, int N, int K,
                         int act, hipStream_t s, int variant = 0, float* skws = nullptr,
                         int sk = 1);
// Residual epilogue: X (ld = N) += acc + bias; X fp32, or fp16 when resid16
// (fp16 compute only: the reference's fp16 GPU residual stream).
hipError_t gemm_residual(int dtype, const void* A, const void* W, const float* bias, void* X,
                         int M, int N, int K, hipStream_t s, int variant = 0, int resid16 = 0,
                         float* skws = nullptr, int sk = 1);
// Float epilogue: C (fp32, ld = N) = acc + bias (bias may be null).
hipError_t gemm_f32(int dtype, const void* A, const void* W, const float* bias, float* C,
                    int M, int N, int K, hipStream_t s, int variant = 0);
// Diagnostic epilogue that writes nothing (prices the epilogue in A/B timing).
hipError_t gemm_null(int dtype, const void* A, const void* W, float* C, int M, int N, int K,
                     hipStream_t s, int variant = 0);
// Patch-embed epilogue: row m = b*np + p of the patch GEMM goes to token row
// b*(np+1) + 1 + p of X (fp32, or fp16 when resid16; ld = N), plus positional
// embedding row 1 + p.
hipError_t gemm_patch(int dtype, const void* A, const void* W, const float* pos, void* X,
                      int M, int N, int K, int np, hipStream_t s, int resid16 = 0);

// ---- MX-fp8 (OCP e4m3 + E8M0 per 32 k) operands and GEMM (gemm_mx.hip) ----
// Scale plane bytes of a [rows, K] operand (tiled, see mx_scale_index).
size_t mx_scale_bytes(int rows, int K);
// Rows [R, K] (fp32, or fp16 when in_f16; K % 256 == 0) -> data q [R, K] bytes + scales sc.
hipError_t quant_mx(int in_f16, const void* in, int R, int K, void* q, void* sc, hipStream_t s);
// C = A[M,K] . W[N,K]^T with MX-fp8 operands (N % 256 == 0, K % 128 == 0).
// epi 0: C fp16 = act(acc + bias); epi 1: C fp16 residual += acc + bias;
// epi 5: C MX-fp8 data [M, N] + scale plane CS = MX(act(acc + bias)).
// variant: 0 persistent where it applies (K >= 256), 1 one tile per workgroup,
// 2 persistent only (bit-identical kernels; A/B)
hipError_t gemm_mx(const void* A, const void* SA, const void* W, const void* SW, const float* bias,
                   void* C, void* CS, int M, int N, int K, int epi, int act, hipStream_t s,
                   int variant = 0);

// ---- LayerNorm (fp32 statistics, eps 1e-5) over rows of width D ----
// Row r of the input is at in + in_row(r)*D with in_row(r) = rows ? rows[r] : r*in_stride_rows;
// the input is fp32, or fp16 when in16 (fp16 residual stream).
// out_f32 != null -> fp32 output (may alias an fp32 in); else out_t in compute dtype (may
// alias an fp16 in of the same dtype).
// normalize != 0 additionally L2-normalises each output row (F.normalize, eps 1e-12).
// out_q != null: MX-fp8 output instead (data out_q [R, D] bytes + tiled scale plane
// out_s, the fp8 GEMM's A operand).
hipError_t layernorm(int dtype, const void* in, const int32_t* rows, int in_stride_rows,
                     const float* gamma, const float* beta, float* out_f32, void* out_t,
                     int R, int D, int normalize, hipStream_t s, int in16 = 0,
                     void* out_q = nullptr, void* out_s = nullptr);

// Row statistics of the fp16 residual stream for the folded LayerNorm: stats[r] =
// {mean, rstd * *rscale} of row r of in [R, D], mean and rstd exactly as layernorm
// computes them; rscale (device, nullable = 1) is the weight's 1/S from ln_fold.
hipError_t ln_stats(const void* in, float* stats, int R, int D, hipStream_t s,
                    const float* rscale = nullptr);
// Fold LayerNorm (gamma, beta) into the following Linear (W [N, K] compute dtype,
// bias [N] fp32 or null): Wf = W diag(gamma) * S (compute dtype), colsum[j] = sum_k Wf[j,k],
// c[j] = bias[j] + sum_k beta[k] W[j,k] (sums in double, fixed order). S is the power
// of two that puts max|W gamma| S in [2^14, 2^15] (no fp16 subnormals for small
// gamma); inv_scale (device float[2], nullable = no scaling) receives 1/S in [0].
hipError_t ln_fold(int dtype, const void* W, const float* gamma, const float* beta,
                   const float* bias, void* Wf, float* colsum, float* c, int N, int K,
                   hipStream_t s, float* inv_scale = nullptr);

// ---- fused multi-head attention over a packed QKV buffer ----
// qkv: [B*N, 3*H*dh] compute dtype (torch in_proj order q|k|v); out: [B*N, H*dh].
// head dim dh = 64 (OpenAI CLIP) or 80 (open_clip ViT-H/14 vision tower; one head
// per workgroup); causal adds the -inf strictly-upper-triangular mask
// (clip/model.py:323-329). variant (dh 64): 0 = default (the two-workgroup x8
// kernel for N in 256..259, else the pipelined multi-head kernel when N <= 320,
// one head per workgroup above), 1 = one head per workgroup, 2 = pipelined,
// 4 = pipelined + last-chunk split, 8 = x8, 10-16 = one head per workgroup on
// that many waves (probe). variant (dh 80): 0 = default (the two-phase kernel where
// it applies), 1 = attention_kernel<80>, 2 = two-phase.
hipError_t attention(int dtype, const void* qkv, void* out, int B, int N, int H, int causal,
                     hipStream_t s, int variant = 0, int head_dim = 64);

// Attention of token row 0 (CLS) of every image only: out [B, H*dh] compact
// (row b = image b's CLS row), same qkv layout; N <= 768, dh 64 or 80 (0 = 64).
hipError_t attention_q0(int dtype, const void* qkv, void* out, int B, int N, int H,
                        hipStream_t s, int head_dim = 64);

// ---- embeddings / gathers ----
// dst[r, :] = src[r * stride_rows, :], rows of D elements of elt_bytes (2 or 4)
hipError_t gather_rows(const void* src, void* dst, int R, int stride_rows, int D, int elt_bytes,
                       hipStream_t s);
// images [B,3,R,R] (in_dtype: kIn32 fp32, kF16, kBF16) -> patches [B*g*g, Kp] compute
// dtype, col = c*P*P + ky*P + kx, zero-padded up to Kp (multiple of 64). variant 0:
// one workgroup per band of patches (vector loads) where R % 4 == 0, 1: one per patch.
hipError_t im2col(int dtype, int in_dtype, const void* img, void* patches, int B, int R, int P,
                  int Kp, hipStream_t s, int variant = 0);
// Clock probe: n_wg one-wave workgroups each store {HW_REG_XCC_ID, s_memtime,
// s_memrealtime, 0} (4 x u64) to out[4 * blockIdx.x ..].
hipError_t clock_probe(unsigned long long* out, int n_wg, hipStream_t s);
// X[b*ntok + 0, :] = cls + pos[0, :]  (X fp32, or fp16 when resid16)
hipError_t class_token(const float* cls, const float* pos, void* X, int B, int ntok, int D,
                       hipStream_t s, int resid16 = 0);
// X[p*L + t, :] = tok_emb[tokens[p*L + t], :] + pos[t, :]; eot[p] = argmax_t tokens[p*L+t]
// as a row index p*L + argmax (first maximum, like torch.argmax). X fp32 / fp16 (resid16).
hipError_t token_embed(const int64_t* tokens, const float* tok_emb, const float* pos, void* X,
                       int32_t* eot_rows, int P, int L, int D, int vocab, hipStream_t s,
                       int resid16 = 0);
// out[r, :] = in[r, :] @ Wm  (fp32 on the f32 MFMA, Wm [D, E] row-major, D % 16 == 0)
hipError_t rowvec_matmul(const float* in, const float* Wm, float* out, int R, int D, int E,
                         hipStream_t s);
// fp32 [rows, src_cols] -> compute dtype [rows, cols] (cols >= src_cols, zero pad), RNE
hipError_t cast_pad(int dtype, const float* in, void* out, int64_t rows, int src_cols, int cols,
                    hipStream_t s);
// in-place row L2 normalisation (F.normalize, eps 1e-12), fp32 [R, D]
hipError_t row_l2norm(float* x, int R, int D, hipStream_t s);
// zero-shot head: f = normalize(x @ proj) (proj may be null -> f = normalize(x));
// logits = scale * f @ tw ([E, C], E % 16 == 0) on the f32 MFMA with the row norm
// fused (head_logits_kernel); topk indices (sorted, largest first; topk_rows_kernel).
// With proj, scratch (fp32 [B, E]) receives the projection, which runs first as
// a chip-wide f32-MFMA kernel (head_proj_kernel, also behind rowvec_matmul).
hipError_t zero_shot(const float* x, const float* proj, const float* tw, float* logits,
                     int32_t* topk, int B, int Din, int E, int C, float scale, int k,
                     hipStream_t s, float* scratch = nullptr);

// ---- cached-feature consumers (outlier scoring), fp32 ----
// norms[r] = ||x[r]||; out = x / max(norms, eps) per row.
hipError_t row_norms(const float* x, int N, int D, float* norms, hipStream_t s);
hipError_t div_rows(const float* x, const float* norms, int N, int D, float eps, float* out,
                    hipStream_t s);
// class k's rows are order[offsets[k] .. offsets[k+1]) (ascending sample order);
// sums [K,D] = per-class sums in that order; centroids = normalize(sums / count).
hipError_t class_centroids(const float* x, const int32_t* order, const int32_t* offsets, int K,
                           int D, float eps, float* sums, float* centroids, hipStream_t s);
// sim[s,p] = (x[s] . protos[p]) * inv_nx[s] * inv_np[p] (null -> 1); per sample:
// own_best / own_arg = max / first argmax over p with owner[p] == cls[s],
// other_best = max over the other prototypes (-inf when none).
hipError_t proto_scores(const float* x, const float* protos, const int32_t* owner,
                        const int32_t* cls, const float* inv_nx, const float* inv_np, int N,
                        int P, int D, float* own_best, int32_t* own_arg, float* other_best,
                        hipStream_t s);

// ---- on-device CLIP preprocessing (bicubic resize + center crop + normalise) ----
// PreCache: geometry-table cache + image-array buffers, one per model handle.
// descs: HOST array of B descriptors (validated, copied stream-ordered);
// out_kind 0 = float32 [B,3,n,n] normalised, 1 = uint8 [B,n,n,3]. On error
// fills `err`.
struct PreCache;
PreCache* pre_cache_create();
void pre_cache_destroy(PreCache* c);
hipError_t preprocess(PreCache* c, const uint8_t* pixels, const miclip_image_desc* descs, int B,
                      int n, int out_kind, void* out, hipStream_t s, char* err, int errlen);

}  // namespace miclip
