/*
 * miclip.h -- C ABI of the MI355X-native CLIP encode path (libmiclip.so).
 *
 * The reference (WhiteGiveFive/aihab-clip) is pure Python and has no FFI; its
 * hot path is the PyTorch call chain behind `clip.load` / `model.encode_image`
 * / `model.encode_text` and the zero-shot head. Each entry point below states
 * the reference interface it replaces (paths relative to the reference repo).
 *
 * Conventions
 *   - Plain pointers and sizes only. Image/token/feature/logit buffers are
 *     caller-owned DEVICE pointers on the handle's device (e.g. torch tensors'
 *     data_ptr()); weights and workspaces are handle-owned.
 *   - Every call is stream-ordered on the caller's `stream` (a hipStream_t;
 *     NULL = the legacy default stream). No call synchronises the device,
 *     except miclip_model_load_weights / miclip_reserve, which allocate.
 *   - Return value: 0 on success, a negative MICLIP_E* code on failure; the
 *     message is available from miclip_last_error() (thread-local).
 *   - A handle is bound to one device and is not safe for concurrent calls
 *     from several host threads.
 */
#ifndef MICLIP_H_
#define MICLIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MICLIP_ABI_VERSION 9

enum miclip_status {
  MICLIP_OK = 0,
  MICLIP_EINVAL = -1,   /* bad argument / shape (reference raises ValueError / RuntimeError) */
  MICLIP_EHIP = -2,     /* HIP runtime error */
  MICLIP_ENOWEIGHTS = -3, /* a tower's weights were not loaded */
  MICLIP_ENOMEM = -4
};

/* MICLIP_MXFP8: the vision tower's QKV, out-proj, c_fc and c_proj on OCP MX-fp8
 * operands (e4m3 + an E8M0 scale per 32 k; weights quantised at load, activations
 * by the producing kernels), the rest -- the whole text tower included -- as
 * MICLIP_FP16. SURVEY §8f row 4 (C5 fp8 weights); parity unpinned. */
/* MICLIP_F32: an input element type only (miclip_encode_image_ex images). */
enum miclip_dtype { MICLIP_FP16 = 0, MICLIP_BF16 = 1, MICLIP_MXFP8 = 2, MICLIP_F32 = 3 };
/* MICLIP_ACT_GELU_TANH: GELU's tanh form, accepted by the op-level MX-fp8 GEMM
 * (miclip_op_gemm_mx epi 5) -- the model's MX c_fc uses it where its output is
 * quantised to e4m3; a model config's act is QUICKGELU or GELU */
enum miclip_act { MICLIP_ACT_QUICKGELU = 1, MICLIP_ACT_GELU = 2, MICLIP_ACT_GELU_TANH = 3 };

/* encode_image flags */
#define MICLIP_FLAG_NORMALIZE 1u  /* F.normalize(feats, dim=-1): aihab_utils/feature_cache.py:126-127 */
#define MICLIP_FLAG_APPLY_PROJ 2u /* feats @ visual.proj:       methods/ProLIP.py:38-41 */
/* miclip_encode_image_ex only: `out` holds fp16 (or bf16) features, the fp32
 * result rounded once (RNE) -- the element type of the reference's GPU path
 * (clip.load on cuda keeps the model fp16, so encode_image returns fp16 and the
 * cached f{v}.pth / embeddings.pt are fp16: aihab_utils/feature_cache.py:126-131,
 * 208-222). The two exclude each other. */
#define MICLIP_FLAG_OUT_FP16 4u
#define MICLIP_FLAG_OUT_BF16 8u

/* Model hyper-parameters; the fields of clip/model.py:240-254 (CLIP.__init__),
 * as inferred by build_model (clip/model.py:396-419). ViT towers only. */
typedef struct miclip_config {
  int32_t embed_dim;
  int32_t image_resolution;
  int32_t vision_layers;
  int32_t vision_width;
  int32_t vision_patch_size;
  int32_t context_length;
  int32_t vocab_size;
  int32_t transformer_width;
  int32_t transformer_heads;
  int32_t transformer_layers;
  int32_t compute_dtype; /* miclip_dtype: GEMM/attention operand type (fp32 accumulate) */
  int32_t act;           /* miclip_act: QuickGELU (clip/model.py:160-162) or exact GELU */
  int32_t vision_head_dim; /* 0 or 64: heads = width // 64 (clip/model.py:268); 80: open_clip
                              ViT-H/14 (16 heads of 80 on width 1280) */
  uint32_t options;        /* MICLIP_OPT_* bits (ABI 7); 0 = the default numerics path */
} miclip_config;

/* Numerics options of a model handle (miclip_config.options). Every path that
 * changes what the kernels compute is chosen here, explicitly -- the library
 * reads no environment variables.
 * RESID_F32: fp32 residual stream (default: fp16 under fp16 AND bf16 compute --
 *   the reference's GPU model keeps its residual stream in half; bf16 compute then
 *   rounds only the GEMM / attention operands to bf16). NO_LN_FOLD: run ln_1 / ln_2
 *   as LayerNorm kernels (default under fp16 compute: folded into the QKV / c_fc
 *   GEMMs on the fp16 stream; bf16 compute never folds: the GEMM would read the fp16
 *   stream as its bf16 operand).
 * MX_OUT_FP16 (MICLIP_MXFP8): keep the vision out-projection fp16 (default MX-fp8).
 * MX_GELU_ERF (MICLIP_MXFP8): exact-erf GELU in the MX c_fc epilogue (default: the
 *   tanh form, <= 4.8e-4 from erf, below the e4m3 step).
 * FULL_LAST_BLOCK: run the last vision block over every token row (default: the
 *   CLS rows only after its QKV GEMM, the only rows ln_post reads, clip/model.py:
 *   226-229); switchable at run time with miclip_model_set_option. */
#define MICLIP_OPT_RESID_F32 1u
#define MICLIP_OPT_NO_LN_FOLD 2u
#define MICLIP_OPT_MX_OUT_FP16 4u
#define MICLIP_OPT_MX_GELU_ERF 8u
#define MICLIP_OPT_FULL_LAST_BLOCK 16u

/* One host fp32 tensor of a CLIP state dict, named as in CLIP.state_dict(). */
typedef struct miclip_tensor {
  const char* name;
  const float* data; /* host, contiguous fp32 */
  int64_t numel;
} miclip_tensor;

typedef struct miclip_model miclip_model;

/* Replaces the construction half of clip.load (clip/clip.py:89-137) /
 * build_model (clip/model.py:396-433): creates an empty model on `device`. */
int miclip_model_create(const miclip_config* cfg, int device, miclip_model** out);

/* Replaces model.load_state_dict + convert_weights (clip/model.py:372-393, 432):
 * copies/repacks the named tensors into handle-owned device memory (GEMM
 * weights in the compute dtype, LayerNorm/bias/embeddings fp32). May be called
 * several times; unknown names are an error, "logit_scale" is accepted and unused. */
int miclip_model_load_weights(miclip_model* m, const miclip_tensor* tensors, int32_t n);
/* Same, with every `data` a DEVICE pointer (fp32, contiguous, on the handle's
 * device): e.g. the model's own torch Parameters after .to(device), so a device
 * move never round-trips the state dict through host memory. Repacking (cast to
 * the compute dtype, conv1 padding, MX quantisation) runs on the device. */
int miclip_model_load_weights_device(miclip_model* m, const miclip_tensor* tensors, int32_t n);

/* Pre-allocates workspaces for up to max_images images / max_prompts prompts,
 * so later encode calls allocate nothing (required before hipGraph capture). */
int miclip_reserve(miclip_model* m, int32_t max_images, int32_t max_prompts);

/* Replaces CLIP.encode_image -> VisionTransformer.forward (clip/model.py:335-336,
 * 216-235). images: device fp32 [B,3,R,R] (CLIP-normalised, clip/clip.py:80).
 * out: device fp32 [B, vision_width] pre-projection features (the modified
 * reference returns ln_post(x[:,0,:]) without @proj, clip/model.py:228-235), or
 * [B, embed_dim] with MICLIP_FLAG_APPLY_PROJ; MICLIP_FLAG_NORMALIZE L2-normalises.
 * fp32 out only (the OUT_FP16 / OUT_BF16 flags are miclip_encode_image_ex's). */
int miclip_encode_image(miclip_model* m, const float* images, int32_t B, float* out,
                        uint32_t flags, void* stream);

/* miclip_encode_image with the input batch's element type named:
 * image_dtype MICLIP_F32, MICLIP_FP16 or MICLIP_BF16 (a device-resident half
 * batch, e.g. the reference's `images.to(device).half()` under clip.load on GPU,
 * clip/model.py:336 `image.type(self.dtype)`, read directly by the patchify:
 * half the input bytes of fp32). Same outputs and flags, plus MICLIP_FLAG_OUT_FP16 /
 * MICLIP_FLAG_OUT_BF16: `out` is then [B, dim] 2-byte elements. Unknown flag
 * bits: MICLIP_EINVAL. */
int miclip_encode_image_ex(miclip_model* m, const void* images, int32_t image_dtype, int32_t B,
                           void* out, uint32_t flags, void* stream);

/* Replaces CLIP.encode_text (clip/model.py:338-353), which returns the tuple
 * (x_before_proj [P, transformer_width], x [P, embed_dim]). tokens: device
 * int64 [P, context_length] as produced by clip.tokenize (clip/clip.py:192-228);
 * EOT row = first argmax of each row. Either output may be NULL. */
int miclip_encode_text(miclip_model* m, const int64_t* tokens, int32_t P, float* x_before,
                       float* x_proj, void* stream);

/* Replaces the zero-shot head of ProLIP eval / compute_image_features_test:
 * f = F.normalize(feats @ visual.proj) (apply_proj != 0) or F.normalize(feats);
 * logits = scale * f @ text_weights  (methods/ProLIP.py:38-41, 288-291;
 * methods/utils.py:181-186; scale 100 in the reference); topk = logits.topk(k)
 * indices, sorted (methods/utils.py:16-21). feats: device fp32 [B, Din];
 * text_weights: device fp32 [embed_dim, C] (clip_classifier output, utils.py:54);
 * logits: device fp32 [B, C]; topk: device int32 [B, k] or NULL. */
int miclip_zero_shot(miclip_model* m, const float* feats, int32_t B, int32_t apply_proj,
                     const float* text_weights, int32_t C, float scale, float* logits,
                     int32_t* topk, int32_t k, void* stream);

/* One decoded image in device memory: interleaved HWC uint8 ('RGB' or 'L'). */
typedef struct miclip_image_desc {
  int64_t offset;     /* byte offset of pixel (0, 0) from the `pixels` base */
  int32_t height;
  int32_t width;
  int32_t channels;   /* 3 (RGB) or 1 (L; replicated to RGB like convert("RGB")) */
  int32_t row_stride; /* bytes between rows; 0 = width * channels */
} miclip_image_desc;

enum miclip_pre_out {
  MICLIP_PRE_F32 = 0, /* float32 [B, 3, R, R], ToTensor + Normalize(CLIP_MEAN, CLIP_STD) */
  MICLIP_PRE_U8 = 1   /* uint8 [B, R, R, 3], the resized + center-cropped RGB pixels */
};

/* On-device CLIP preprocessing, R = the model's image_resolution. Replaces the
 * per-image CPU transform of clip/clip.py:74-81 (`_transform`) and
 * data/clip_transforms.py:50-55 (test split): Resize(R, BICUBIC) of the shorter
 * side -> CenterCrop(R) -> RGB -> ToTensor -> Normalize; bit-exact with
 * Pillow's resize (libImaging/Resample.c) and torchvision's size/anchor rules.
 * pixels: device uint8 base; descs: HOST array [B] (copied, stream-ordered,
 * into a handle-owned device buffer before return); out: device, see
 * miclip_pre_out. Images may differ in size (ragged batch). Errors: EINVAL for
 * a bad descriptor or a downscale beyond 64 taps (about 16x at R = 224). */
int miclip_preprocess(miclip_model* m, const uint8_t* pixels, const miclip_image_desc* descs,
                      int32_t B, void* out, int32_t out_kind, void* stream);

/* ---- cached-feature consumers: outlier scoring, fp32 ----
 * Replace the torch ops of tools/outlier_cleaning.py's scorers on the
 * embeddings cache; all pointers are device memory, calls stream-ordered.
 * miclip_row_norms: norms[N] = emb.norm(dim=-1) (outlier_cleaning.py:234);
 * with out != NULL also out = emb / max(norms, eps) (:244). */
int miclip_row_norms(const float* x, int32_t N, int32_t D, float* norms, float eps, float* out,
                     void* stream);
/* Per-class normalised centroids (compute_centroids, :266-276): class k's
 * rows are order[offsets[k] .. offsets[k+1]) in ascending sample order (a
 * stable sort of the labels), summed in that order -- bit-identical to the
 * CPU index_add_ -- then means = sums / count, F.normalize(eps).
 * sums: scratch [K, D]; centroids: [K, D]. */
int miclip_class_centroids(const float* x, const int32_t* order, const int32_t* offsets,
                           int32_t K, int32_t D, float eps, float* sums, float* centroids,
                           void* stream);
/* Nearest-prototype scores (score_prototype_distance, :626-673; with inverse
 * norms the cosine of score_centroid_distance, :329): sim = x . proto *
 * inv_nx[s] * inv_np[p] (either may be NULL = 1); own_best / own_arg = best
 * similarity and first best prototype index among owner[p] == cls[s];
 * other_best = best over the other prototypes (-inf when there are none). */
int miclip_proto_scores(const float* x, const float* protos, const int32_t* owner,
                        const int32_t* cls, const float* inv_nx, const float* inv_np, int32_t N,
                        int32_t P, int32_t D, float* own_best, int32_t* own_arg,
                        float* other_best, void* stream);

/* Batch split of encode_image over the caller's stream and one handle-owned
 * stream (fork/join by events, so the call stays stream-ordered and
 * graph-capturable): 1 = off, 2..4 = that many parts (default 2; a part is
 * never smaller than 16 images). */
int miclip_set_splits(miclip_model* m, int32_t splits);
/* Parts encode_image splits a batch of B images into (>= 1): at most the
 * miclip_set_splits value, no part below 16 images or 16384 token rows. */
int miclip_image_splits(const miclip_model* m, int32_t B);

/* Diagnostics (no reference counterpart; SURVEY §8d measurement): n_wg one-wave
 * workgroups each write {XCD id (HW_REG_XCC_ID), s_memtime (shader-clock
 * counter), s_memrealtime (100 MHz), 0} as 4 uint64 to device out[4*i..].
 * Launched before and after a timed region on its stream, the per-XCD ratio of
 * the two counters' deltas is the core clock the chip held over that region. */
int miclip_clock_probe(uint64_t* out, int32_t n_wg, void* stream);

void miclip_model_destroy(miclip_model* m);
const char* miclip_last_error(void);
int miclip_abi_version(void);
/* Device-memory bytes currently held by the handle (weights + workspaces). */
int64_t miclip_model_bytes(const miclip_model* m);
/* Numerics path the handle runs (from miclip_config.options and the dtype):
 * MICLIP_MODEL_RESID16 fp16 residual stream, MICLIP_MODEL_LNFOLD ln_1 / ln_2 folded
 * into the vision tower's QKV / c_fc GEMMs (MICLIP_MODEL_LNFOLD_TEXT: the text
 * tower's; MX-fp8 models fold the text tower only), MICLIP_MODEL_MXFP8 MX-fp8 GEMM
 * operands (vision tower),
 * MICLIP_MODEL_CLS_LAST last vision block on the CLS rows, MICLIP_MODEL_MX_OUT MX-fp8
 * vision out-projection, MICLIP_MODEL_MX_GELU_TANH tanh-form GELU in the MX c_fc
 * epilogue. 0 for NULL. */
#define MICLIP_MODEL_RESID16 1
#define MICLIP_MODEL_LNFOLD 2
#define MICLIP_MODEL_MXFP8 4
#define MICLIP_MODEL_CLS_LAST 8
#define MICLIP_MODEL_MX_OUT 16
#define MICLIP_MODEL_MX_GELU_TANH 32
#define MICLIP_MODEL_LNFOLD_TEXT 64
int miclip_model_flags(const miclip_model* m);
/* Diagnostics: the GEMM kernel of the block launches (>= 256 rows) --
 * which 0: the folded-LN store GEMMs (QKV, c_fc), 1: the fp16 residual GEMMs
 * (out-proj, c_proj); variant 0 (default) / 259 (the 8-wave persistent kernel);
 * which 2: the MX-fp8 GEMMs (variants of miclip_op_gemm_mx_v). All are
 * bit-identical, so results never change;
 * bench.py --ab-gemm times them in one process. */
int miclip_set_gemm_variant(miclip_model* m, int32_t which, int32_t variant);
/* Switches a run-time option of a handle (only MICLIP_OPT_FULL_LAST_BLOCK; the
 * others fix the weight layout at create and return MICLIP_EINVAL). */
int miclip_model_set_option(miclip_model* m, uint32_t option, int32_t on);

/* ---- diagnostics: per-kernel-class timing with HIP events ---- */

/* Algorithmic totals of one kernel class since the last reset. `flops` counts
 * 2*M*N*K per GEMM and 4*N^2*dh per attention head; `bytes` is the minimum HBM
 * traffic (operands read once, outputs written once). */
typedef struct miclip_kernel_stat {
  const char* name;
  int64_t launches;
  double ms;
  double flops;
  double bytes;
} miclip_kernel_stat;

/* When enabled, every launch of later encode calls is bracketed by hipEvents on
 * the caller's stream (adds a few us per launch: use outside timed regions). */
int miclip_set_profiling(miclip_model* m, int enable);
/* Synchronises on the recorded events, folds them into per-class totals and
 * copies up to n classes into out; returns the number of classes. */
int miclip_profile_read(miclip_model* m, miclip_kernel_stat* out, int32_t n, int32_t reset);

/* ---- op-level entry points (kernel parity tests and micro-benchmarks) ---- */

/* C = A[M,K] . W[N,K]^T + bias, A/W in compute dtype `dtype`.
 * epi 0: C dtype = act(.) with act from `act` (0 none); epi 1: C fp32 += (residual);
 * epi 2: C fp32 = . ; epi 3: no output (diagnostic: prices the epilogue);
 * epi 4: C fp16 += . (fp16 residual stream; dtype MICLIP_FP16 only).
 * N % 128 == 0 and K % 64 == 0 required. variant: 0 = tile
 * chosen by size, 128 / 256 = force the 128x128 / 256x256 kernel (N % 256 for 256);
 * 259 = the persistent 256-row-tile kernel; 192 / 129 / 130 = its 192-row tiles /
 * 128-row tiles / 128-row tiles + row tail (epi 0 and 4 only; N % 256, K >= 128).
 * 259 / 192 / 129 / 130 give bit-identical results (same k order and epilogue per row).
 * Replaces torch Linear (clip/model.py:171-175) and MHA in/out projections. */
int miclip_op_gemm(int32_t dtype, const void* A, const void* W, const float* bias, void* C,
                   int32_t M, int32_t N, int32_t K, int32_t epi, int32_t act, int32_t variant,
                   void* stream);

/* Folded LayerNorm (ln_1 -> QKV, ln_2 -> c_fc of ResidualAttentionBlock,
 * clip/model.py:184-185): LN(x) . W^T + b computed as rs * (x . Wf^T - mean * colsum) + c
 * with rs = rstd / S.
 * miclip_op_ln_fold: Wf = W diag(gamma) * S (dtype), colsum = row sums of Wf, c = bias + W beta
 *   (W [N, K] dtype; gamma, beta [K], bias [N] fp32, bias may be null). S is the power of
 *   two that puts max|W gamma| S in [2^14, 2^15], so a small gamma never rounds W gamma into
 *   the fp16 subnormals; inv_scale: device float[2] ([0] receives 1/S, [1] is scratch), or
 *   NULL for S = 1.
 * miclip_op_ln_stats: stats[r] = {mean, rstd * *rscale} (fp32 pairs) of the fp16 rows
 *   x [R, D]; rscale = the fold's inv_scale (device), or NULL for 1.
 * miclip_op_gemm_ln: C [M, N] (dtype) = act(rs * (A . Wf^T - mean * colsum) + c), A [M, K]
 *   the un-normalised rows (act as miclip_op_gemm; variant as there). */
/* The split-K GEMM of the CLS-only last vision block (gemm_nt_splitk_kernel +
 * splitk_reduce_kernel), op level: sk K slices (K % (64 sk) == 0) summed in
 * ascending order through ws (device fp32, >= sk * M * N floats), then the epilogue.
 * epi 0: C dtype = act(. + bias); 1: C fp32 += . + bias; 4: C fp16 += . + bias (the
 * fp16 residual stream); 5: the folded-LN store of miclip_op_gemm_ln (c, colsum,
 * stats; act). N % 128 == 0. Replaces the CLS rows' Linear calls (clip/model.py:
 * 171-175, 179-181 on ln_post's rows, :226-229). */
int miclip_op_gemm_splitk(int32_t dtype, const void* A, const void* W, const float* bias,
                          const float* c, const float* colsum, const float* stats, void* C,
                          int32_t M, int32_t N, int32_t K, int32_t epi, int32_t act, int32_t sk,
                          float* ws, void* stream);
int miclip_op_ln_stats(const void* x, float* stats, int32_t R, int32_t D, const float* rscale,
                       void* stream);
int miclip_op_ln_fold(int32_t dtype, const void* W, const float* gamma, const float* beta,
                      const float* bias, void* Wf, float* colsum, float* c, int32_t N, int32_t K,
                      float* inv_scale, void* stream);
int miclip_op_gemm_ln(int32_t dtype, const void* A, const void* Wf, const float* c,
                      const float* colsum, const float* stats, void* C, int32_t M, int32_t N,
                      int32_t K, int32_t act, int32_t variant, void* stream);

/* LayerNorm over R rows of width D (eps 1e-5, fp32 statistics); replaces the
 * reference LayerNorm (clip/model.py:151-157). flags bit 0: out fp32 (else compute
 * dtype); bit 1: in fp16 (the fp16 residual stream; dtype MICLIP_FP16 only), else fp32. */
int miclip_op_layernorm(int32_t dtype, const void* in, const float* gamma, const float* beta,
                        void* out, int32_t flags, int32_t R, int32_t D, void* stream);

/* softmax(Q K^T / sqrt(dh) + mask) V per head over a packed qkv [B*N, 3*H*dh]
 * buffer, out [B*N, H*dh]; replaces F.scaled_dot_product_attention inside
 * nn.MultiheadAttention (clip/model.py:179-181), causal = text mask (323-329).
 * head_dim dh: 64, or 80 (open_clip ViT-H/14 vision tower); 0 means 64.
 * variant (dh 64): 0 = default (two workgroups per CU at N = 256..259, else the
 * pipelined multi-head kernel for N <= 320, else one head per workgroup), 1 = one
 * head per workgroup, 2 = pipelined, 4 = pipelined with the last-chunk split,
 * 8 = two workgroups per CU, 10..16 = one head per workgroup on that many waves.
 * variant (dh 80): 0 = default (6 at N = 256..259, else 2 where it applies, else
 * 1), 1 = one head per workgroup (N <= 416), 2 = two-phase fetch (N = 160..288),
 * 6 = pipelined half-head K/V ring (N = 256..259). A variant outside its range
 * fails (never silently replaced). */
int miclip_op_attention(int32_t dtype, const void* qkv, void* out, int32_t B, int32_t N,
                        int32_t H, int32_t head_dim, int32_t causal, int32_t variant,
                        void* stream);

/* conv1 patchify as the patch GEMM's A operand (clip/model.py:217-219): images
 * [B, 3, R, R] (image_dtype MICLIP_F32 / FP16 / BF16) -> patches [B*(R/P)^2, Kp]
 * (dtype FP16 / BF16), column c*P*P + ky*P + kx, zero up to Kp (>= 3*P*P). variant 0 =
 * default (one workgroup per band of R/P patches -- 16-B vector loads and stores -- where
 * R % 4 == 0, Kp % 4 == 0 and `images` and `patches` are 16-byte aligned, else 1), 1 = one
 * workgroup per patch (element accesses, no alignment requirement). Bit-identical. The
 * encode entry points take any alignment the same way. */
int miclip_op_im2col(int32_t dtype, int32_t image_dtype, const void* images, void* patches,
                     int32_t B, int32_t R, int32_t P, int32_t Kp, int32_t variant, void* stream);

/* Attention of the first query (token row 0, CLS) of every image only, same qkv
 * layout as miclip_op_attention; out [B, H*dh] compact (row b = image b's CLS
 * row). The vision tower's last block (only its CLS rows reach ln_post,
 * clip/model.py:226-229). N <= 768, dh 64 or 80 (0 = 64), non-causal. */
int miclip_op_attention_q0(int32_t dtype, const void* qkv, void* out, int32_t B, int32_t N,
                           int32_t H, int32_t head_dim, void* stream);

/* ---- MX-fp8 operands (MICLIP_MXFP8; no reference counterpart: C5 stretch) ----
 * An MX-fp8 [rows, K] operand is e4m3 bytes [rows, K] plus a tiled E8M0 scale
 * plane of miclip_mx_scale_bytes(rows, K) bytes (one scale per 32 consecutive k). */
int64_t miclip_mx_scale_bytes(int32_t rows, int32_t K);
/* rows [R, K] (in_f16: 0 fp32, 1 fp16, 2 fp16 through the older 8-lane-block
 * kernel -- byte-identical, kept for that test; K % 256 == 0) -> q [R, K] + scales */
int miclip_op_quant_mx(const void* in, int32_t in_f16, int32_t R, int32_t K, void* q, void* scales,
                       void* stream);
/* C = A . W^T on MX-fp8 operands (N % 256 == 0, K % 128 == 0). epi 0: C fp16 =
 * act(. + bias); epi 1: C fp16 += . + bias; epi 5: C MX-fp8 (+ CS scales) = MX(act(. + bias)). */
int miclip_op_gemm_mx(const void* A, const void* SA, const void* W, const void* SW,
                      const float* bias, void* C, void* CS, int32_t M, int32_t N, int32_t K,
                      int32_t epi, int32_t act, void* stream);
/* miclip_op_gemm_mx with the kernel named: variant 0 default (persistent where K >=
 * 256), 1 one 256x256 tile per workgroup, 2 persistent (MICLIP_EINVAL where it does
 * not apply). Bit-identical outputs (A/B and tests). */
int miclip_op_gemm_mx_v(const void* A, const void* SA, const void* W, const void* SW,
                        const float* bias, void* C, void* CS, int32_t M, int32_t N, int32_t K,
                        int32_t epi, int32_t act, int32_t variant, void* stream);
/* LayerNorm (fp32 in, or fp16 if in_f16) -> MX-fp8 rows q [R, D] + scales */
int miclip_op_layernorm_mx(const void* in, int32_t in_f16, const float* gamma, const float* beta,
                           void* q, void* scales, int32_t R, int32_t D, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MICLIP_H_ */
