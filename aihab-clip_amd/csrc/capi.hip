// C ABI of libmiclip.so (declared in include/miclip.h): model handle, weight
// repacking, workspaces, and the encode_image / encode_text / zero-shot
// orchestration over the CDNA4 kernels.
//
// Forward schedule of one ResidualAttentionBlock (clip/model.py:183-186), with
// the residual stream x kept in fp32 [B*N, W] (token-major, i.e. NLD: the
// reference's LND permutes (clip/model.py:224-226) are a layout choice that
// does not change per-token arithmetic):
//   h   = LN1(x)                           layernorm      -> compute dtype
//   qkv = h . Wqkv^T + b                   gemm_store     [M, 3W]
//   o   = MHA core(qkv)                    attention      [M, W]
//   x  += o . Wo^T + bo                    gemm_residual
//   h   = LN2(x)                           layernorm
//   f   = QuickGELU(h . Wfc^T + bfc)       gemm_store     [M, 4W]
//   x  += f . Wp^T + bp                    gemm_residual
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/miclip.h"
#include "common.h"
#include "kernels.h"

using namespace miclip;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define MICLIP_HIP(expr)                                                                 \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return fail(_e == hipErrorInvalidValue ? MICLIP_EINVAL : MICLIP_EHIP,              \
                  std::string(#expr) + ": " + hipGetErrorString(_e));                    \
  } while (0)

uint16_t f32_to_bf16_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

uint16_t f32_to_f16_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t b;
  std::memcpy(&b, &h, 2);
  return b;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct Block {
  void* w_qkv = nullptr;
  float* b_qkv = nullptr;
  void* w_out = nullptr;
  float* b_out = nullptr;
  void* w_fc = nullptr;
  float* b_fc = nullptr;
  void* w_proj = nullptr;
  float* b_proj = nullptr;
  float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
  // MX-fp8 models: scale planes of w_qkv / w_fc / w_proj (which then hold e4m3 bytes)
  void *s_qkv = nullptr, *s_fc = nullptr, *s_proj = nullptr, *s_out = nullptr;
  // folded LayerNorm (miclip_model::lnfold): W diag(gamma) of QKV / c_fc, their
  // column sums and folded biases (epilogue.h EpiStoreLN)
  void *wf_qkv = nullptr, *wf_fc = nullptr;
  float *cs_qkv = nullptr, *c_qkv = nullptr, *cs_fc = nullptr, *c_fc = nullptr;
  float *fs_qkv = nullptr, *fs_fc = nullptr;   // [2] each: 1/S of the fold (ln_stats rscale)
};

struct Workspace {
  int cap_rows = 0;   // token rows
  int cap_items = 0;  // images or prompts
  void* patches = nullptr;
  void* x = nullptr;  // residual stream: fp32, or fp16 (miclip_model::resid16)
  void* h = nullptr;
  void* qkv = nullptr;
  void* o = nullptr;
  void* f = nullptr;
  // MX-fp8 models: LayerNorm output (hq, scales hs) and c_fc output (fq, fs)
  void *hq = nullptr, *hs = nullptr, *fq = nullptr, *fs = nullptr;
  void* xc = nullptr;     // [items, W] the CLS rows of x (last vision block, run_block)
  float* feat = nullptr;  // [items, W] fp32 scratch
  int32_t* rows = nullptr;
  float* stats = nullptr;  // [rows] {mean, rstd} for the folded LayerNorm
};

}  // namespace

struct miclip_model {
  miclip_config cfg{};
  int device = 0;
  int dtype = 0;
  // fp16 residual stream (x between blocks), the reference's own fp16 GPU model
  // (clip.load on cuda: convert_weights, clip/model.py:372-393, and the half
  // activations of VisionTransformer / Transformer). Default under fp16 and bf16
  // compute; MICLIP_OPT_RESID_F32 keeps an fp32 stream.
  int resid16 = 0;
  // MICLIP_MXFP8: the vision tower's QKV / c_fc / c_proj run on MX-fp8 operands
  // (gemm_mx.hip); everything else (patch embed, attention, the text tower) as
  // fp16 compute.
  bool mx = false;
  // MX-fp8 models: the VISION tower's attention out-projection on MX-fp8 too (the
  // attention output quantised by quant_mx: 80-wide heads straddle the 32-wide
  // blocks, so no attention epilogue can); MICLIP_OPT_MX_OUT_FP16 keeps it fp16.
  // Image 1-cos moved 4.90e-4 -> 4.96e-4 for +1.0 % (C5, same box:
  // profiles/r03/configs/mx_out_ab.txt)
  bool mx_out = false;
  // MX c_fc epilogue: GELU in its tanh form (default) or exact erf
  // (MICLIP_OPT_MX_GELU_ERF); see mx_act
  bool mx_gelu_erf = false;
  // the last vision block on the CLS rows only (default; MICLIP_OPT_FULL_LAST_BLOCK
  // clears it, also at run time: miclip_model_set_option)
  bool cls_last = true;
  // GEMM kernel variants for the full-batch launches (M >= 16384 rows), set by
  // miclip_set_gemm_variant for same-process A/B: [0] the folded-LN store GEMMs
  // (QKV, c_fc), [1] the fp16 residual GEMMs (out-proj, c_proj). 0 = default.
  // Only variants bit-identical to the default are accepted: results never change.
  int gemm_variant[3] = {0, 0, 0};   // [2]: the MX-fp8 GEMMs (gemm_mx variant)
  // ln_1 / ln_2 folded into the QKV / c_fc GEMMs (fp16 stream models;
  // MICLIP_OPT_NO_LN_FOLD runs the LayerNorm kernels instead); folded weights are
  // rebuilt per tower after every weight load
  int lnfold = 0;
  bool folded[2] = {false, false};   // [visual, text]
  int Kp = 0;  // padded patch-GEMM K
  std::unordered_map<void*, size_t> allocs;
  int64_t bytes = 0;
  // tensor name -> (device pointer, numel, kind)
  struct Slot {
    void** dst;
    int64_t numel;
    int kind;  // 0 = fp32 as-is, 1 = GEMM weight in compute dtype, 2 = conv1 -> [W, Kp]
    bool loaded;
    bool visual;
    void** sdst = nullptr;  // MX-fp8 weight: its scale plane (dst then holds e4m3 bytes)
  };
  std::unordered_map<std::string, Slot> slots;
  std::vector<Block> vblocks, tblocks;
  void* conv_w = nullptr;
  float *cls = nullptr, *vpos = nullptr, *ln_pre_g = nullptr, *ln_pre_b = nullptr;
  float *ln_post_g = nullptr, *ln_post_b = nullptr, *vproj = nullptr;
  float *tok_emb = nullptr, *tpos = nullptr, *ln_final_g = nullptr, *ln_final_b = nullptr;
  float* text_proj = nullptr;
  float* logit_scale = nullptr;
  Workspace wimg, wtxt;
  int splits = 2;               // batch split over the caller stream + aux (miclip_set_splits)
  hipStream_t aux[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
  // per-kernel-class HIP-event timing (miclip_set_profiling)
  struct ProfRec {
    int cls;
    hipEvent_t a, b;
    double flops, bytes;
  };
  bool profiling = false;
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> event_pool;
  struct ProfAcc {
    int64_t launches = 0;
    double ms = 0, flops = 0, bytes = 0;
  };
  std::vector<ProfAcc> prof_acc;
  PreCache* pre = nullptr;   // miclip_preprocess state (geometry tables, image array)
  float* zs_scratch = nullptr;   // zero-shot projected rows [B, embed_dim]
  int64_t zs_cap = 0;
};

namespace {

// K_CLS_BLOCK: everything of the last vision block after its QKV GEMM, on the
// CLS rows only (run_block cls_only)
enum KClass {
  K_IM2COL, K_GEMM_PATCH, K_LAYERNORM, K_GEMM_QKV, K_ATTENTION, K_GEMM_OUT, K_GEMM_FC,
  K_GEMM_PROJ, K_HEAD, K_TEXT_EMBED, K_CLS_BLOCK, K_ZERO_SHOT, K_NUM
};
const char* const kClassNames[K_NUM] = {"im2col", "gemm_patch", "layernorm", "gemm_qkv",
                                        "attention", "gemm_out", "gemm_fc", "gemm_proj",
                                        "head", "text_embed", "cls_block", "zero_shot"};

hipEvent_t take_event(miclip_model* m) {
  if (!m->event_pool.empty()) {
    hipEvent_t e = m->event_pool.back();
    m->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Brackets one launch with events when profiling is on (outside timed runs).
struct ProfScope {
  miclip_model* m;
  int cls;
  hipStream_t s;
  double flops, bytes;
  hipEvent_t a = nullptr;
  ProfScope(miclip_model* m_, int c, hipStream_t s_, double f, double b)
      : m(m_), cls(c), s(s_), flops(f), bytes(b) {
    if (m->profiling && (a = take_event(m))) (void)hipEventRecord(a, s);
  }
  ~ProfScope() {
    if (!a) return;
    hipEvent_t b = take_event(m);
    if (!b) return;
    (void)hipEventRecord(b, s);
    m->pending.push_back({cls, a, b, flops, bytes});
  }
};

int elt() { return 2; }

void add_slot(miclip_model* m, const std::string& name, void** dst, int64_t numel, int kind,
              bool visual, void** sdst = nullptr) {
  m->slots[name] = miclip_model::Slot{dst, numel, kind, false, visual, sdst};
}

void add_block_slots(miclip_model* m, const std::string& prefix, Block& b, int W, bool visual) {
  // MX-fp8 operands in the VISION tower only: the text tower is one classifier's
  // prompts per run (no throughput reason for fp8), and on MX its 1-cos was
  // 4.5e-3 against the north star's 1e-3, so it runs the fp16 kernels
  const bool mx = m->mx && visual;
  add_slot(m, prefix + "attn.in_proj_weight", &b.w_qkv, (int64_t)3 * W * W, 1, visual,
           mx ? &b.s_qkv : nullptr);
  add_slot(m, prefix + "attn.in_proj_bias", (void**)&b.b_qkv, 3 * W, 0, visual);
  add_slot(m, prefix + "attn.out_proj.weight", &b.w_out, (int64_t)W * W, 1, visual,
           m->mx_out && visual ? &b.s_out : nullptr);
  add_slot(m, prefix + "attn.out_proj.bias", (void**)&b.b_out, W, 0, visual);
  add_slot(m, prefix + "ln_1.weight", (void**)&b.ln1_g, W, 0, visual);
  add_slot(m, prefix + "ln_1.bias", (void**)&b.ln1_b, W, 0, visual);
  add_slot(m, prefix + "mlp.c_fc.weight", &b.w_fc, (int64_t)4 * W * W, 1, visual,
           mx ? &b.s_fc : nullptr);
  add_slot(m, prefix + "mlp.c_fc.bias", (void**)&b.b_fc, 4 * W, 0, visual);
  add_slot(m, prefix + "mlp.c_proj.weight", &b.w_proj, (int64_t)4 * W * W, 1, visual,
           mx ? &b.s_proj : nullptr);
  add_slot(m, prefix + "mlp.c_proj.bias", (void**)&b.b_proj, W, 0, visual);
  add_slot(m, prefix + "ln_2.weight", (void**)&b.ln2_g, W, 0, visual);
  add_slot(m, prefix + "ln_2.bias", (void**)&b.ln2_b, W, 0, visual);
}

int dev_alloc(miclip_model* m, void** p, size_t bytes) {
  MICLIP_HIP(hipMalloc(p, bytes));
  m->allocs[*p] = bytes;
  m->bytes += (int64_t)bytes;
  return 0;
}

void dev_free(miclip_model* m, void* p) {
  if (!p) return;
  auto it = m->allocs.find(p);
  if (it != m->allocs.end()) {
    m->bytes -= (int64_t)it->second;
    m->allocs.erase(it);
  }
  (void)hipFree(p);
}

bool tower_loaded(const miclip_model* m, bool visual) {
  for (const auto& kv : m->slots)
    if (kv.second.visual == visual && !kv.second.loaded && kv.first != "logit_scale")
      return false;
  return true;
}

std::string missing(const miclip_model* m, bool visual) {
  for (const auto& kv : m->slots)
    if (kv.second.visual == visual && !kv.second.loaded && kv.first != "logit_scale")
      return kv.first;
  return "";
}

int ensure_ws(miclip_model* m, Workspace& w, int items, int ntok, int W, bool image) {
  if (items <= w.cap_items) return 0;
  const int rows = items * ntok;
  const size_t e = elt();
  // grow: make sure no queued kernel still uses the old buffers
  MICLIP_HIP(hipDeviceSynchronize());
  for (void* p : {w.patches, (void*)w.x, w.h, w.qkv, w.o, w.f, w.hq, w.hs, w.fq, w.fs, w.xc,
                  (void*)w.feat, (void*)w.rows, (void*)w.stats})
    dev_free(m, p);
  w = Workspace{};
  int rc;
  if (image) {
    const int g = m->cfg.image_resolution / m->cfg.vision_patch_size;
    if ((rc = dev_alloc(m, &w.patches, (size_t)items * g * g * m->Kp * e))) return rc;
  }
  if ((rc = dev_alloc(m, &w.x, (size_t)rows * W * (m->resid16 ? 2 : 4)))) return rc;
  // h (the LayerNorm output) is unused when ln_1 / ln_2 are folded into the GEMMs
  if (!m->lnfold && (rc = dev_alloc(m, &w.h, (size_t)rows * W * e))) return rc;
  if ((rc = dev_alloc(m, &w.qkv, (size_t)rows * 3 * W * e))) return rc;
  if ((rc = dev_alloc(m, &w.o, (size_t)rows * W * e))) return rc;
  if ((rc = dev_alloc(m, &w.f, (size_t)rows * 4 * W * e))) return rc;
  if (m->mx && image) {
    // scale planes: + 4 blocks of 256 rows so that every batch-split window
    // (view) starts on its own 256-row block
    if ((rc = dev_alloc(m, &w.hq, (size_t)rows * W))) return rc;
    if ((rc = dev_alloc(m, &w.hs, mx_scale_bytes(rows + 4 * 256, W)))) return rc;
    if ((rc = dev_alloc(m, &w.fq, (size_t)rows * 4 * W))) return rc;
    if ((rc = dev_alloc(m, &w.fs, mx_scale_bytes(rows + 4 * 256, 4 * W)))) return rc;
  }
  if ((rc = dev_alloc(m, &w.xc, (size_t)items * W * (m->resid16 ? 2 : 4)))) return rc;
  if ((rc = dev_alloc(m, (void**)&w.feat, (size_t)items * W * 4))) return rc;
  if ((rc = dev_alloc(m, (void**)&w.rows, (size_t)items * 4))) return rc;
  if ((rc = dev_alloc(m, (void**)&w.stats, (size_t)rows * 8))) return rc;
  w.cap_items = items;
  w.cap_rows = rows;
  return 0;
}

// Algorithmic cost of one GEMM launch: 2MNK flops; bytes = read A and W once,
// write C (2 B/elt), plus the fp32 residual read+write for residual epilogues.
double gemm_flops(double M, double N, double K) { return 2.0 * M * N * K; }
double gemm_bytes(double M, double N, double K, double c_bytes) {
  return 2.0 * M * K + 2.0 * N * K + c_bytes * M * N;
}

// Build the folded QKV / c_fc weights of one tower (after every weight load).
int ensure_folded(miclip_model* m, bool visual) {
  // an MX model's vision tower quantises the LayerNorm output instead (run_block)
  if (!m->lnfold || (visual && m->mx) || m->folded[visual ? 0 : 1]) return 0;
  const int W = visual ? m->cfg.vision_width : m->cfg.transformer_width;
  int rc;
  for (Block& b : visual ? m->vblocks : m->tblocks) {
    if (!b.wf_qkv) {
      if ((rc = dev_alloc(m, &b.wf_qkv, (size_t)3 * W * W * elt()))) return rc;
      if ((rc = dev_alloc(m, &b.wf_fc, (size_t)4 * W * W * elt()))) return rc;
      if ((rc = dev_alloc(m, (void**)&b.cs_qkv, (size_t)3 * W * 4))) return rc;
      if ((rc = dev_alloc(m, (void**)&b.c_qkv, (size_t)3 * W * 4))) return rc;
      if ((rc = dev_alloc(m, (void**)&b.cs_fc, (size_t)4 * W * 4))) return rc;
      if ((rc = dev_alloc(m, (void**)&b.c_fc, (size_t)4 * W * 4))) return rc;
      if ((rc = dev_alloc(m, (void**)&b.fs_qkv, 8))) return rc;
      if ((rc = dev_alloc(m, (void**)&b.fs_fc, 8))) return rc;
    }
    MICLIP_HIP(ln_fold(m->dtype, b.w_qkv, b.ln1_g, b.ln1_b, b.b_qkv, b.wf_qkv, b.cs_qkv, b.c_qkv,
                       3 * W, W, nullptr, b.fs_qkv));
    MICLIP_HIP(ln_fold(m->dtype, b.w_fc, b.ln2_g, b.ln2_b, b.b_fc, b.wf_fc, b.cs_fc, b.c_fc,
                       4 * W, W, nullptr, b.fs_fc));
  }
  MICLIP_HIP(hipDeviceSynchronize());
  m->folded[visual ? 0 : 1] = true;
  return 0;
}

// One ResidualAttentionBlock (clip/model.py:183-186) over items x N token rows.
// cls_only (the vision tower's last block): VisionTransformer.forward keeps only
// ln_post(x[:, 0, :]) of its output (clip/model.py:226-229), so after the QKV
// GEMM over all rows (every token's key and value) only the CLS query is
// attended (attention_q0) and out-proj, ln_2 and the MLP run on the items CLS
// rows, gathered into the compact residual block w.xc. Row for row these are the
// same operations as the full block (GEMM rows are independent; the tile and row-
// tail paths round alike), so the CLS features are those of the full block up to
// the attention's summation order.
// Activation of the MX-fp8 c_fc epilogue, whose output is quantised to e4m3 for
// c_proj: exact GELU (open_clip's nn.GELU) runs in its tanh form there -- its
// <= 4.8e-4 deviation (2e-4 relative) is far below the e4m3 step (2^-3), and it issues ~9
// fewer packed VALU ops per element pair than the erf fit (c_fc 0.68 -> 0.59 ms at
// M = 65792, profiles/r03/configs/mx_epi.jsonl). MICLIP_OPT_MX_GELU_ERF keeps erf.
int mx_act(const miclip_model* m, int act) {
  return act == ACT_GELU && !m->mx_gelu_erf ? ACT_GELU_TANH : act;
}

// Split count of a CLS-row GEMM (M = images) reducing K: slices of >= 256 k, at most
// 16, dividing K into whole 64-k steps. A function of K only, so a row's result
// never depends on the batch.
int cls_splitk(int K) {
  int sk = K / 256 < 16 ? K / 256 : 16;
  while (sk > 1 && K % (sk * 64)) --sk;
  return sk < 1 ? 1 : sk;
}

int run_block(miclip_model* m, const Block& b, Workspace& w, int items, int N, int W, int H,
              int dh, int causal, hipStream_t s, bool cls_only = false) {
  const int M = items * N, dt = m->dtype, r16 = m->resid16;
  const int vln = M >= 256 ? m->gemm_variant[0] : 0;
  const int vres = M >= 256 ? m->gemm_variant[1] : 0;
  const double dM = M, dW = W, rb = r16 ? 2 : 4;  // residual bytes per element
  const bool mx = b.s_qkv != nullptr;   // MX-fp8 operands for QKV / c_fc / c_proj (vision)
  const bool fold = m->lnfold && b.wf_qkv;
  if (fold) {
    ProfScope p(m, K_LAYERNORM, s, 0, dM * (dW * rb + 8));
    MICLIP_HIP(ln_stats(w.x, w.stats, M, W, s, b.fs_qkv));
  } else {
    ProfScope p(m, K_LAYERNORM, s, 0, dM * dW * (rb + (mx ? 1 : 2)));
    if (mx)
      MICLIP_HIP(layernorm(dt, w.x, nullptr, 1, b.ln1_g, b.ln1_b, nullptr, nullptr, M, W, 0, s,
                           r16, w.hq, w.hs));
    else
      MICLIP_HIP(
          layernorm(dt, w.x, nullptr, 1, b.ln1_g, b.ln1_b, nullptr, w.h, M, W, 0, s, r16));
  }
  {
    ProfScope p(m, K_GEMM_QKV, s, gemm_flops(dM, 3 * dW, dW), gemm_bytes(dM, 3 * dW, dW, 2));
    if (mx)
      MICLIP_HIP(gemm_mx(w.hq, w.hs, b.w_qkv, b.s_qkv, b.b_qkv, w.qkv, nullptr, M, 3 * W, W, 0,
                         ACT_NONE, s, m->gemm_variant[2]));
    else if (fold)
      MICLIP_HIP(gemm_store_ln(dt, w.x, b.wf_qkv, b.c_qkv, b.cs_qkv, w.stats, w.qkv, M, 3 * W, W,
                               ACT_NONE, s, vln));
    else
      MICLIP_HIP(gemm_store(dt, w.h, b.w_qkv, b.b_qkv, w.qkv, M, 3 * W, W, ACT_NONE, s));
  }
  if (cls_only) {
    const double dI = items;
    ProfScope p(m, K_CLS_BLOCK, s,
                4.0 * dI * H * N * dh + gemm_flops(dI, dW, dW) + gemm_flops(dI, 4 * dW, dW) +
                    gemm_flops(dI, dW, 4 * dW),
                dM * 2 * dW * 2 + 10 * dW * dW * 2);
    MICLIP_HIP(attention_q0(dt, w.qkv, w.o, items, N, H, s, dh));
    MICLIP_HIP(gather_rows(w.x, w.xc, items, N, W, r16 ? 2 : 4, s));
    // the GEMMs below have M = images: split K through an fp32 workspace in the
    // QKV buffer (free after attention_q0; sk * items * 4W floats fit in its
    // items * N * 3W elements for N >= 43 tokens)
    float* skws = (float*)w.qkv;
    const bool sk_ok = (size_t)16 * 4 * W * 4 <= (size_t)N * 3 * W * elt();
    const int sk1 = sk_ok ? cls_splitk(W) : 1, sk4 = sk_ok ? cls_splitk(4 * W) : 1;
    if (b.s_out) {   // MX-fp8 out-proj (vision tower of an MX model)
      MICLIP_HIP(quant_mx(1, w.o, items, W, w.hq, w.hs, s));
      MICLIP_HIP(gemm_mx(w.hq, w.hs, b.w_out, b.s_out, b.b_out, w.xc, nullptr, items, W, W, 1,
                         ACT_NONE, s, m->gemm_variant[2]));
    } else {
      MICLIP_HIP(gemm_residual(dt, w.o, b.w_out, b.b_out, w.xc, items, W, W, s, 0, r16, skws,
                               sk1));
    }
    if (mx) {   // MX-fp8 MLP on the CLS rows (their scale blocks are row-local)
      MICLIP_HIP(layernorm(dt, w.xc, nullptr, 1, b.ln2_g, b.ln2_b, nullptr, nullptr, items, W, 0,
                           s, r16, w.hq, w.hs));
      MICLIP_HIP(gemm_mx(w.hq, w.hs, b.w_fc, b.s_fc, b.b_fc, w.fq, w.fs, items, 4 * W, W, 5,
                         mx_act(m, m->cfg.act), s, m->gemm_variant[2]));
      MICLIP_HIP(gemm_mx(w.fq, w.fs, b.w_proj, b.s_proj, b.b_proj, w.xc, nullptr, items, W, 4 * W,
                         1, ACT_NONE, s, m->gemm_variant[2]));
      return 0;
    }
    if (fold) {
      MICLIP_HIP(ln_stats(w.xc, w.stats, items, W, s, b.fs_fc));
      MICLIP_HIP(gemm_store_ln(dt, w.xc, b.wf_fc, b.c_fc, b.cs_fc, w.stats, w.f, items, 4 * W, W,
                               m->cfg.act, s, 0, skws, sk1));
    } else {
      MICLIP_HIP(
          layernorm(dt, w.xc, nullptr, 1, b.ln2_g, b.ln2_b, nullptr, w.h, items, W, 0, s, r16));
      MICLIP_HIP(gemm_store(dt, w.h, b.w_fc, b.b_fc, w.f, items, 4 * W, W, m->cfg.act, s, 0, skws,
                            sk1));
    }
    MICLIP_HIP(gemm_residual(dt, w.f, b.w_proj, b.b_proj, w.xc, items, W, 4 * W, s, 0, r16, skws,
                             sk4));
    return 0;
  }
  {
    const double n = N;
    ProfScope p(m, K_ATTENTION, s, 4.0 * items * H * n * n * dh, dM * dW * 2 * 4);
    MICLIP_HIP(attention(dt, w.qkv, w.o, items, N, H, causal, s, 0, dh));
  }
  {
    ProfScope p(m, K_GEMM_OUT, s, gemm_flops(dM, dW, dW), gemm_bytes(dM, dW, dW, 2 * rb));
    if (b.s_out) {   // quantise the attention output (hq / hs are free here), MX GEMM
      MICLIP_HIP(quant_mx(1, w.o, M, W, w.hq, w.hs, s));
      MICLIP_HIP(gemm_mx(w.hq, w.hs, b.w_out, b.s_out, b.b_out, w.x, nullptr, M, W, W, 1,
                         ACT_NONE, s, m->gemm_variant[2]));
    } else {
      MICLIP_HIP(gemm_residual(dt, w.o, b.w_out, b.b_out, w.x, M, W, W, s, r16 ? vres : 0, r16));
    }
  }
  if (fold) {
    ProfScope p(m, K_LAYERNORM, s, 0, dM * (dW * rb + 8));
    MICLIP_HIP(ln_stats(w.x, w.stats, M, W, s, b.fs_fc));
  } else {
    ProfScope p(m, K_LAYERNORM, s, 0, dM * dW * (rb + (mx ? 1 : 2)));
    if (mx)
      MICLIP_HIP(layernorm(dt, w.x, nullptr, 1, b.ln2_g, b.ln2_b, nullptr, nullptr, M, W, 0, s,
                           r16, w.hq, w.hs));
    else
      MICLIP_HIP(
          layernorm(dt, w.x, nullptr, 1, b.ln2_g, b.ln2_b, nullptr, w.h, M, W, 0, s, r16));
  }
  {
    ProfScope p(m, K_GEMM_FC, s, gemm_flops(dM, 4 * dW, dW),
                mx ? dM * dW + 4 * dW * dW + 4 * dM * dW : gemm_bytes(dM, 4 * dW, dW, 2));
    if (mx)
      MICLIP_HIP(gemm_mx(w.hq, w.hs, b.w_fc, b.s_fc, b.b_fc, w.fq, w.fs, M, 4 * W, W, 5,
                         mx_act(m, m->cfg.act), s, m->gemm_variant[2]));
    else if (fold)
      MICLIP_HIP(gemm_store_ln(dt, w.x, b.wf_fc, b.c_fc, b.cs_fc, w.stats, w.f, M, 4 * W, W,
                               m->cfg.act, s, vln));
    else
      MICLIP_HIP(gemm_store(dt, w.h, b.w_fc, b.b_fc, w.f, M, 4 * W, W, m->cfg.act, s));
  }
  {
    ProfScope p(m, K_GEMM_PROJ, s, gemm_flops(dM, dW, 4 * dW),
                mx ? 4 * dM * dW + 4 * dW * dW + 2 * rb * dM * dW
                   : gemm_bytes(dM, dW, 4 * dW, 2 * rb));
    if (mx)
      MICLIP_HIP(gemm_mx(w.fq, w.fs, b.w_proj, b.s_proj, b.b_proj, w.x, nullptr, M, W, 4 * W, 1,
                         ACT_NONE, s, m->gemm_variant[2]));
    else
      MICLIP_HIP(gemm_residual(dt, w.f, b.w_proj, b.b_proj, w.x, M, W, 4 * W, s, r16 ? vres : 0,
                               r16));
  }
  return 0;
}

// A window of the workspace: rows [row0, ...) / items [item0, ...).
Workspace view(const miclip_model* m, const Workspace& w, size_t row0, size_t item0, int N,
               int W, int part = 0) {
  Workspace v = w;
  const size_t e = elt();
  const int g = m->cfg.image_resolution / m->cfg.vision_patch_size;
  if (w.patches) v.patches = (char*)w.patches + item0 * g * g * m->Kp * e;
  v.x = (char*)w.x + row0 * W * (m->resid16 ? 2 : 4);
  if (w.h) v.h = (char*)w.h + row0 * W * e;
  v.qkv = (char*)w.qkv + row0 * 3 * W * e;
  v.o = (char*)w.o + row0 * W * e;
  v.f = (char*)w.f + row0 * 4 * W * e;
  if (w.hq) {
    // window `part` starts its scale planes at 256-row block ceil(row0/256) + part:
    // ceil(a) + ceil(b) <= ceil(a + b) + 1, so windows never share a block
    const size_t blk = (row0 + 255) / 256 + part;
    v.hq = (char*)w.hq + row0 * W;
    v.fq = (char*)w.fq + row0 * 4 * W;
    v.hs = (char*)w.hs + blk * (W / 128) * 1024;
    v.fs = (char*)w.fs + blk * (4 * W / 128) * 1024;
  }
  v.xc = (char*)w.xc + item0 * W * (m->resid16 ? 2 : 4);
  v.feat = w.feat + item0 * W;
  v.rows = w.rows + item0;
  v.stats = w.stats + 2 * row0;
  (void)N;
  return v;
}

int ensure_aux(miclip_model* m, int n) {
  if (!m->ev_fork) MICLIP_HIP(hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming));
  for (int i = 0; i < n && i < 3; ++i) {
    if (!m->aux[i]) MICLIP_HIP(hipStreamCreateWithFlags(&m->aux[i], hipStreamNonBlocking));
    if (!m->ev_join[i]) MICLIP_HIP(hipEventCreateWithFlags(&m->ev_join[i], hipEventDisableTiming));
  }
  return 0;
}

// encode_image for B images whose workspace window is `w` (clip/model.py:216-235)
int encode_image_part(miclip_model* m, Workspace w, const void* images, int in_dt, int B,
                      void* out, uint32_t flags, hipStream_t s) {
  const auto& c = m->cfg;
  const int P = c.vision_patch_size, R = c.image_resolution, W = c.vision_width;
  const int dh = c.vision_head_dim, g = R / P, np = g * g, N = np + 1, H = W / dh;
  const int dt = m->dtype;
  const int M = B * N;
  int rc;
  {
    ProfScope p(m, K_IM2COL, s, 0,
                (double)B * 3 * R * R * (in_dt == kIn32 ? 4 : 2) + (double)B * np * m->Kp * 2);
    MICLIP_HIP(im2col(dt, in_dt, images, w.patches, B, R, P, m->Kp, s));
  }
  {
    const double dM = (double)B * np;
    const int rb = m->resid16 ? 2 : 4;
    ProfScope p(m, K_GEMM_PATCH, s, gemm_flops(dM, W, 3.0 * P * P),
                gemm_bytes(dM, W, m->Kp, rb));
    MICLIP_HIP(gemm_patch(dt, w.patches, m->conv_w, m->vpos, w.x, B * np, W, m->Kp, np, s,
                          m->resid16));
  }
  {
    ProfScope p(m, K_LAYERNORM, s, 0, (double)M * W * (m->resid16 ? 4 : 8));
    MICLIP_HIP(class_token(m->cls, m->vpos, w.x, B, N, W, s, m->resid16));
    // ln_pre in place: fp32 stream -> fp32 out; fp16 stream -> compute-dtype (fp16) out
    MICLIP_HIP(layernorm(m->resid16 ? kF16 : dt, w.x, nullptr, 1, m->ln_pre_g, m->ln_pre_b,
                         m->resid16 ? nullptr : (float*)w.x, m->resid16 ? w.x : nullptr, M, W,
                         0, s, m->resid16));
  }
  // the last block on the CLS rows only (run_block); N beyond attention_q0's
  // range (never for CLIP's towers) runs it whole
  const bool cls_last = m->cls_last && N <= 768;
  for (int l = 0; l < c.vision_layers; ++l)
    if ((rc = run_block(m, m->vblocks[l], w, B, N, W, H, dh, 0, s,
                        cls_last && l == c.vision_layers - 1)))
      return rc;
  const bool proj = flags & MICLIP_FLAG_APPLY_PROJ, norm = flags & MICLIP_FLAG_NORMALIZE;
  // ln_post on the CLS rows only (clip/model.py:228): rows b*N of x, or the
  // compact CLS block xc
  const void* xcls = cls_last ? w.xc : w.x;
  const int cstride = cls_last ? 1 : N;
  // half-precision features (MICLIP_FLAG_OUT_FP16 / _BF16, the reference's fp16
  // f{v}.pth files): the fp32 head result, rounded once (RNE) into `out`; the
  // fp32 result goes through the c_fc buffer, free by now
  const int odt = (flags & MICLIP_FLAG_OUT_FP16) ? kF16 : (flags & MICLIP_FLAG_OUT_BF16) ? kBF16 : -1;
  float* o32 = odt < 0 ? (float*)out : proj ? (float*)w.f : w.feat;
  const int dim = proj ? c.embed_dim : W;
  ProfScope p(m, K_HEAD, s, proj ? 2.0 * B * W * c.embed_dim : 0.0, (double)B * W * 8);
  if (!proj) {
    MICLIP_HIP(layernorm(dt, xcls, nullptr, cstride, m->ln_post_g, m->ln_post_b, o32, nullptr, B,
                         W, norm ? 1 : 0, s, m->resid16));
  } else {
    MICLIP_HIP(layernorm(dt, xcls, nullptr, cstride, m->ln_post_g, m->ln_post_b, w.feat, nullptr,
                         B, W, 0, s, m->resid16));
    MICLIP_HIP(rowvec_matmul(w.feat, m->vproj, o32, B, W, c.embed_dim, s));
    if (norm) MICLIP_HIP(row_l2norm(o32, B, c.embed_dim, s));
  }
  if (odt >= 0) MICLIP_HIP(cast_pad(odt, o32, out, B, dim, dim, s));
  return 0;
}

bool cfg_ok(const miclip_config& c, std::string& why) {
  auto bad = [&](const char* w) { why = w; return false; };
  if (c.vision_width % 256 || c.vision_width < 256 || c.vision_width > 1536)
    return bad("vision_width must be a multiple of 256 in [256, 1536]");
  if (c.transformer_width % 256 || c.transformer_width < 256 || c.transformer_width > 1536)
    return bad("transformer_width must be a multiple of 256 in [256, 1536]");
  if (c.transformer_heads * 64 != c.transformer_width)
    return bad("transformer_heads * 64 must equal transformer_width (head dim 64)");
  if (c.vision_patch_size < 1 || c.image_resolution % c.vision_patch_size)
    return bad("image_resolution must be a multiple of vision_patch_size");
  if (c.vision_head_dim != 64 && c.vision_head_dim != 80)
    return bad("vision_head_dim must be 64 or 80");
  if (c.vision_width % c.vision_head_dim) return bad("vision_width % vision_head_dim != 0");
  const int g = c.image_resolution / c.vision_patch_size;
  // K and V images of one head in LDS: 128-B rows (dh 64) / 192-B rows (dh 80)
  const int rowb = c.vision_head_dim == 64 ? 128 : 192;
  if ((g * g + 1 + 31) / 32 * 32 * 2 * rowb > 160 * 1024)
    return bad("too many vision tokens for the attention kernel (max 640 at dh 64, 416 at 80)");
  if (c.context_length < 1 || c.context_length > 640) return bad("context_length out of range");
  if (c.vision_layers < 1 || c.transformer_layers < 0) return bad("bad layer count");
  if (c.embed_dim < 1 || c.vocab_size < 1) return bad("bad embed_dim / vocab_size");
  if (c.compute_dtype != MICLIP_FP16 && c.compute_dtype != MICLIP_BF16 &&
      c.compute_dtype != MICLIP_MXFP8)
    return bad("compute_dtype must be MICLIP_FP16, MICLIP_BF16 or MICLIP_MXFP8");
  if (c.compute_dtype == MICLIP_MXFP8 &&
      (c.vision_width % 256 || c.transformer_width % 256))
    return bad("MICLIP_MXFP8 needs widths that are multiples of 256");
  if (c.act != MICLIP_ACT_QUICKGELU && c.act != MICLIP_ACT_GELU) return bad("bad act");
  if (c.options & ~(MICLIP_OPT_RESID_F32 | MICLIP_OPT_NO_LN_FOLD | MICLIP_OPT_MX_OUT_FP16 |
                    MICLIP_OPT_MX_GELU_ERF | MICLIP_OPT_FULL_LAST_BLOCK))
    return bad("unknown options bits");
  if ((c.options & MICLIP_OPT_RESID_F32) && c.compute_dtype == MICLIP_MXFP8)
    return bad("MICLIP_OPT_RESID_F32 is not available with MICLIP_MXFP8");
  return true;
}

}  // namespace

extern "C" {

const char* miclip_last_error(void) { return g_last_error.c_str(); }
int miclip_abi_version(void) { return MICLIP_ABI_VERSION; }

int miclip_model_create(const miclip_config* cfg, int device, miclip_model** out) {
  if (!cfg || !out) return fail(MICLIP_EINVAL, "null argument");
  std::string why;
  miclip_config c = *cfg;
  if (c.vision_head_dim == 0) c.vision_head_dim = 64;  // ABI v2 callers: zero-filled field
  if (!cfg_ok(c, why)) return fail(MICLIP_EINVAL, "invalid config: " + why);
  int ndev = 0;
  MICLIP_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MICLIP_EINVAL, "invalid device index");
  MICLIP_HIP(hipSetDevice(device));
  auto* m = new miclip_model();
  m->cfg = c;
  m->device = device;
  const uint32_t o = c.options;
  m->mx = cfg->compute_dtype == MICLIP_MXFP8;
  m->mx_out = m->mx && !(o & MICLIP_OPT_MX_OUT_FP16);
  m->mx_gelu_erf = (o & MICLIP_OPT_MX_GELU_ERF) != 0;
  m->cls_last = !(o & MICLIP_OPT_FULL_LAST_BLOCK);
  m->dtype = m->mx ? MICLIP_FP16 : cfg->compute_dtype;   // the fp16 kernels' operand type
  // fp16 stream: every MX model (its text tower's folded path included), fp16
  // compute unless RESID_F32; LN fold on the fp16 stream unless NO_LN_FOLD (MX
  // vision blocks quantise the LayerNorm output instead: run_block)
  m->resid16 = m->mx || !(o & MICLIP_OPT_RESID_F32);
  m->lnfold = m->resid16 && m->dtype == MICLIP_FP16 && !(o & MICLIP_OPT_NO_LN_FOLD);
  const int P = cfg->vision_patch_size, Wv = cfg->vision_width, Wt = cfg->transformer_width;
  m->Kp = (3 * P * P + 63) / 64 * 64;
  const int g = cfg->image_resolution / P, N = g * g + 1, E = cfg->embed_dim;
  m->vblocks.resize(cfg->vision_layers);
  m->tblocks.resize(cfg->transformer_layers);
  add_slot(m, "positional_embedding", (void**)&m->tpos, (int64_t)cfg->context_length * Wt, 0, false);
  add_slot(m, "text_projection", (void**)&m->text_proj, (int64_t)Wt * E, 0, false);
  add_slot(m, "logit_scale", (void**)&m->logit_scale, 1, 0, false);
  add_slot(m, "visual.class_embedding", (void**)&m->cls, Wv, 0, true);
  add_slot(m, "visual.positional_embedding", (void**)&m->vpos, (int64_t)N * Wv, 0, true);
  add_slot(m, "visual.proj", (void**)&m->vproj, (int64_t)Wv * E, 0, true);
  add_slot(m, "visual.conv1.weight", &m->conv_w, (int64_t)Wv * 3 * P * P, 2, true);
  add_slot(m, "visual.ln_pre.weight", (void**)&m->ln_pre_g, Wv, 0, true);
  add_slot(m, "visual.ln_pre.bias", (void**)&m->ln_pre_b, Wv, 0, true);
  add_slot(m, "visual.ln_post.weight", (void**)&m->ln_post_g, Wv, 0, true);
  add_slot(m, "visual.ln_post.bias", (void**)&m->ln_post_b, Wv, 0, true);
  for (int i = 0; i < cfg->vision_layers; ++i)
    add_block_slots(m, "visual.transformer.resblocks." + std::to_string(i) + ".", m->vblocks[i],
                    Wv, true);
  for (int i = 0; i < cfg->transformer_layers; ++i)
    add_block_slots(m, "transformer.resblocks." + std::to_string(i) + ".", m->tblocks[i], Wt,
                    false);
  add_slot(m, "token_embedding.weight", (void**)&m->tok_emb, (int64_t)cfg->vocab_size * Wt, 0,
           false);
  add_slot(m, "ln_final.weight", (void**)&m->ln_final_g, Wt, 0, false);
  add_slot(m, "ln_final.bias", (void**)&m->ln_final_b, Wt, 0, false);
  *out = m;
  return 0;
}

}  // extern "C"

namespace {

// Copies / repacks the named fp32 tensors; `device_src`: t[i].data are device
// pointers on the handle's device (no host round trip), else host pointers.
// GEMM weights are cast (and conv1 padded) on the device from one fp32 staging
// upload -- or straight from the caller's device tensor.
int load_weights(miclip_model* m, const miclip_tensor* t, int32_t n, bool device_src) {
  if (!m || (!t && n)) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(hipSetDevice(m->device));
  m->folded[0] = m->folded[1] = false;
  const hipMemcpyKind kind = device_src ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  void* stage = nullptr;
  size_t stage_bytes = 0;
  auto done = [&](int rc) {
    if (stage) {
      (void)hipDeviceSynchronize();
      dev_free(m, stage);
    }
    return rc;
  };
  // HIP errors leave through done() too: it synchronises before freeing the
  // staging buffer a cast may still be reading
#define LW_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return done(fail(_e == hipErrorInvalidValue ? MICLIP_EINVAL : MICLIP_EHIP,       \
                       std::string(#expr) + ": " + hipGetErrorString(_e)));           \
  } while (0)
  for (int i = 0; i < n; ++i) {
    if (!t[i].name || !t[i].data) return done(fail(MICLIP_EINVAL, "null tensor name/data"));
    auto it = m->slots.find(t[i].name);
    if (it == m->slots.end())
      return done(fail(MICLIP_EINVAL, std::string("unexpected key in state_dict: ") + t[i].name));
    auto& slot = it->second;
    if (t[i].numel != slot.numel)
      return done(fail(MICLIP_EINVAL, std::string("size mismatch for ") + t[i].name + ": got " +
                                          std::to_string(t[i].numel) + ", expected " +
                                          std::to_string(slot.numel)));
    int rc;
    if (slot.kind == 0) {
      if (!*slot.dst && (rc = dev_alloc(m, slot.dst, (size_t)slot.numel * 4))) return done(rc);
      LW_HIP(hipMemcpy(*slot.dst, t[i].data, (size_t)slot.numel * 4, kind));
      slot.loaded = true;
      continue;
    }
    int64_t rows = 0, cols = 0, src_cols = 0;
    if (slot.kind == 1) {
      // nn.Linear / in_proj weight [out, in]: already the W[N][K] operand layout
      const bool is_cproj = it->first.find("c_proj") != std::string::npos;
      const int W = slot.visual ? m->cfg.vision_width : m->cfg.transformer_width;
      cols = is_cproj ? 4 * W : W;
      rows = slot.numel / cols;
      src_cols = cols;
    } else {
      // conv1.weight [W, 3, P, P] -> [W, Kp] zero-padded (col = c*P*P + ky*P + kx)
      const int P = m->cfg.vision_patch_size;
      rows = m->cfg.vision_width;
      src_cols = 3 * P * P;
      cols = m->Kp;
    }
    // fp32 source rows on the device
    const float* src = t[i].data;
    const size_t src_bytes = (size_t)slot.numel * 4;
    if (!device_src) {
      if (src_bytes > stage_bytes) {
        if (stage) {
          LW_HIP(hipDeviceSynchronize());
          dev_free(m, stage);
          stage = nullptr;
        }
        if ((rc = dev_alloc(m, &stage, src_bytes))) return done(rc);
        stage_bytes = src_bytes;
      }
      LW_HIP(hipMemcpy(stage, t[i].data, src_bytes, hipMemcpyHostToDevice));
      src = (const float*)stage;
    }
    if (slot.sdst) {
      // MX-fp8 weight: fp32 rows quantised on the device (quant_mx, gemm_mx.hip)
      const size_t nb = (size_t)rows * cols;
      if (!*slot.dst && (rc = dev_alloc(m, slot.dst, nb))) return done(rc);
      if (!*slot.sdst && (rc = dev_alloc(m, slot.sdst, mx_scale_bytes(rows, cols)))) return done(rc);
      LW_HIP(quant_mx(0, src, (int)rows, (int)cols, *slot.dst, *slot.sdst, nullptr));
    } else {
      if (!*slot.dst && (rc = dev_alloc(m, slot.dst, (size_t)rows * cols * elt()))) return done(rc);
      LW_HIP(cast_pad(m->dtype, src, *slot.dst, rows, (int)src_cols, (int)cols, nullptr));
    }
    // the next upload reuses the staging buffer: finish this conversion first
    if (!device_src) LW_HIP(hipStreamSynchronize(nullptr));
    slot.loaded = true;
  }
  if (device_src) LW_HIP(hipDeviceSynchronize());
  return done(0);
}
#undef LW_HIP

}  // namespace

extern "C" {

int miclip_model_load_weights(miclip_model* m, const miclip_tensor* t, int32_t n) {
  return load_weights(m, t, n, false);
}

int miclip_model_load_weights_device(miclip_model* m, const miclip_tensor* t, int32_t n) {
  return load_weights(m, t, n, true);
}

int miclip_reserve(miclip_model* m, int32_t max_images, int32_t max_prompts) {
  if (!m || max_images < 0 || max_prompts < 0) return fail(MICLIP_EINVAL, "bad argument");
  MICLIP_HIP(hipSetDevice(m->device));
  const int g = m->cfg.image_resolution / m->cfg.vision_patch_size;
  int rc;
  if (max_images &&
      (rc = ensure_ws(m, m->wimg, max_images, g * g + 1, m->cfg.vision_width, true)))
    return rc;
  if (max_prompts && (rc = ensure_ws(m, m->wtxt, max_prompts, m->cfg.context_length,
                                     m->cfg.transformer_width, false)))
    return rc;
  return 0;
}

// Parts the batch of B images (N tokens each) is split into over streams: at
// most m->splits, no part below 16 images, and none below kSplitRows rows. Two
// streams pay wherever the parts keep 16+ images (same-process splits A/B, round
// 6, profiles/r06/splits/): ViT-L/14 at 32 / 64 / 96 images +5.9 / +3.1 / +8.8 %,
// 48 and 128 level, ViT-B/32 bf16 at 256 level (86.5k vs 86.0k img/s; it lost 9 %
// in round 1, before the 192-row tiles); three streams lose 5-15 %.
static int image_splits(const miclip_model* m, int B, int N) {
  constexpr int64_t kSplitRows = 4096;
  int splits = m->profiling ? 1 : m->splits;
  while (splits > 1 && (B < 16 * splits || (int64_t)B * N < kSplitRows * splits)) --splits;
  return splits;
}

int miclip_encode_image(miclip_model* m, const float* images, int32_t B, float* out,
                        uint32_t flags, void* stream) {
  if (flags & (MICLIP_FLAG_OUT_FP16 | MICLIP_FLAG_OUT_BF16))
    return fail(MICLIP_EINVAL, "miclip_encode_image writes fp32 (use miclip_encode_image_ex)");
  return miclip_encode_image_ex(m, images, MICLIP_F32, B, out, flags, stream);
}

int miclip_encode_image_ex(miclip_model* m, const void* images, int32_t image_dtype, int32_t B,
                           void* out, uint32_t flags, void* stream) {
  if (!m || !images || !out || B < 1) return fail(MICLIP_EINVAL, "bad argument to encode_image");
  if (flags & ~(MICLIP_FLAG_NORMALIZE | MICLIP_FLAG_APPLY_PROJ | MICLIP_FLAG_OUT_FP16 |
                MICLIP_FLAG_OUT_BF16))
    return fail(MICLIP_EINVAL, "unknown encode_image flags");
  if ((flags & MICLIP_FLAG_OUT_FP16) && (flags & MICLIP_FLAG_OUT_BF16))
    return fail(MICLIP_EINVAL, "MICLIP_FLAG_OUT_FP16 and MICLIP_FLAG_OUT_BF16 exclude each other");
  const size_t out_bytes = (flags & (MICLIP_FLAG_OUT_FP16 | MICLIP_FLAG_OUT_BF16)) ? 2 : 4;
  if (image_dtype != MICLIP_F32 && image_dtype != MICLIP_FP16 && image_dtype != MICLIP_BF16)
    return fail(MICLIP_EINVAL, "image_dtype must be MICLIP_F32, MICLIP_FP16 or MICLIP_BF16");
  const int in_dt = image_dtype == MICLIP_F32 ? kIn32 : image_dtype == MICLIP_FP16 ? kF16 : kBF16;
  const size_t in_bytes = image_dtype == MICLIP_F32 ? 4 : 2;
  if (!tower_loaded(m, true))
    return fail(MICLIP_ENOWEIGHTS, "visual weights not loaded (missing " + missing(m, true) + ")");
  if (int rc0 = ensure_folded(m, true)) return rc0;
  hipStream_t s = (hipStream_t)stream;
  const auto& c = m->cfg;
  const int R = c.image_resolution, W = c.vision_width;
  const int g = R / c.vision_patch_size, N = g * g + 1;
  int rc;
  if ((rc = ensure_ws(m, m->wimg, B, N, W, true))) return rc;
  const int dim = (flags & MICLIP_FLAG_APPLY_PROJ) ? c.embed_dim : W;
  // Batch split over `splits` streams (caller's + handle-owned aux streams):
  // the parts are independent images, so their kernel sequences overlap (one
  // part's HBM-bound epilogues / LayerNorm / attention run beside another part's
  // MFMA-bound GEMMs, and a GEMM's partial last wave of tiles is filled by
  // another stream's work). Each part uses its own window of the workspace.
  const int splits = image_splits(m, B, N);
  if (splits == 1)
    return encode_image_part(m, view(m, m->wimg, 0, 0, N, W), images, in_dt, B, out, flags, s);
  if ((rc = ensure_aux(m, splits - 1))) return rc;
  MICLIP_HIP(hipEventRecord(m->ev_fork, s));
  int b0 = 0;
  for (int p = 0; p < splits; ++p) {
    const int nb = (B - b0) / (splits - p);
    hipStream_t sp = p == 0 ? s : m->aux[p - 1];
    if (p > 0) MICLIP_HIP(hipStreamWaitEvent(sp, m->ev_fork, 0));
    if ((rc = encode_image_part(m, view(m, m->wimg, (size_t)b0 * N, b0, N, W, p),
                                (const char*)images + (size_t)b0 * 3 * R * R * in_bytes, in_dt,
                                nb, (char*)out + (size_t)b0 * dim * out_bytes, flags, sp)))
      return rc;
    b0 += nb;
  }
  for (int p = 1; p < splits; ++p) {
    MICLIP_HIP(hipEventRecord(m->ev_join[p - 1], m->aux[p - 1]));
    MICLIP_HIP(hipStreamWaitEvent(s, m->ev_join[p - 1], 0));
  }
  return 0;
}

int miclip_image_splits(const miclip_model* m, int32_t B) {
  if (!m || B < 1) return fail(MICLIP_EINVAL, "bad argument to image_splits");
  const int g = m->cfg.image_resolution / m->cfg.vision_patch_size;
  return image_splits(m, B, g * g + 1);
}

int miclip_set_splits(miclip_model* m, int32_t splits) {
  if (!m || splits < 1 || splits > 4) return fail(MICLIP_EINVAL, "splits must be in [1, 4]");
  m->splits = splits;
  return 0;
}

int miclip_encode_text(miclip_model* m, const int64_t* tokens, int32_t P, float* x_before,
                       float* x_proj, void* stream) {
  if (!m || !tokens || P < 1) return fail(MICLIP_EINVAL, "bad argument to encode_text");
  if (!tower_loaded(m, false))
    return fail(MICLIP_ENOWEIGHTS, "text weights not loaded (missing " + missing(m, false) + ")");
  if (int rc0 = ensure_folded(m, false)) return rc0;
  hipStream_t s = (hipStream_t)stream;
  const auto& c = m->cfg;
  const int L = c.context_length, W = c.transformer_width, H = c.transformer_heads;
  int rc;
  if ((rc = ensure_ws(m, m->wtxt, P, L, W, false))) return rc;
  Workspace& w = m->wtxt;
  {
    ProfScope p(m, K_TEXT_EMBED, s, 0, (double)P * L * W * 12);
    MICLIP_HIP(token_embed(tokens, m->tok_emb, m->tpos, w.x, w.rows, P, L, W, c.vocab_size, s,
                           m->resid16));
  }
  for (int l = 0; l < c.transformer_layers; ++l)
    if ((rc = run_block(m, m->tblocks[l], w, P, L, W, H, 64, 1, s))) return rc;
  float* xb = x_before ? x_before : w.feat;
  ProfScope p(m, K_HEAD, s, x_proj ? 2.0 * P * W * c.embed_dim : 0.0, (double)P * W * 8);
  MICLIP_HIP(layernorm(m->dtype, w.x, w.rows, 0, m->ln_final_g, m->ln_final_b, xb, nullptr, P, W,
                       0, s, m->resid16));
  if (x_proj) MICLIP_HIP(rowvec_matmul(xb, m->text_proj, x_proj, P, W, c.embed_dim, s));
  return 0;
}

int miclip_zero_shot(miclip_model* m, const float* feats, int32_t B, int32_t apply_proj,
                     const float* text_weights, int32_t C, float scale, float* logits,
                     int32_t* topk, int32_t k, void* stream) {
  if (!m || !feats || !text_weights || !logits || B < 1 || C < 1 || k < 0 || k > C)
    return fail(MICLIP_EINVAL, "bad argument to zero_shot");
  if (apply_proj && !m->slots["visual.proj"].loaded)
    return fail(MICLIP_ENOWEIGHTS, "visual.proj not loaded");
  const int E = m->cfg.embed_dim;
  const int Din = apply_proj ? m->cfg.vision_width : E;
  if (apply_proj && (int64_t)B * E > m->zs_cap) {
    if (m->zs_scratch) {
      MICLIP_HIP(hipStreamSynchronize((hipStream_t)stream));   // may still be read
      dev_free(m, m->zs_scratch);
      m->zs_scratch = nullptr;
      m->zs_cap = 0;
    }
    const int64_t cap = (int64_t)(B < 256 ? 256 : B) * E;
    if (int rc = dev_alloc(m, (void**)&m->zs_scratch, sizeof(float) * cap)) return rc;
    m->zs_cap = cap;
  }
  ProfScope p(m, K_ZERO_SHOT, (hipStream_t)stream,
              2.0 * B * ((apply_proj ? (double)Din * E : 0.0) + (double)E * C),
              4.0 * ((double)B * Din + (apply_proj ? (double)Din * E : 0.0) + (double)E * C +
                     (double)B * C));
  MICLIP_HIP(zero_shot(feats, apply_proj ? m->vproj : nullptr, text_weights, logits,
                       topk, B, Din, E, C, scale, topk ? k : 0, (hipStream_t)stream,
                       apply_proj ? m->zs_scratch : nullptr));
  return 0;
}

int miclip_preprocess(miclip_model* m, const uint8_t* pixels, const miclip_image_desc* descs,
                      int32_t B, void* out, int32_t out_kind, void* stream) {
  if (!m || !pixels || !descs || !out || B < 1)
    return fail(MICLIP_EINVAL, "bad argument to preprocess");
  if (!m->pre) m->pre = pre_cache_create();
  char err[256] = {0};
  const hipError_t e = preprocess(m->pre, pixels, descs, B, m->cfg.image_resolution, out_kind,
                                  out, (hipStream_t)stream, err, sizeof(err));
  if (e != hipSuccess)
    return fail(e == hipErrorInvalidValue ? MICLIP_EINVAL : MICLIP_EHIP,
                err[0] ? std::string(err) : std::string("preprocess: ") + hipGetErrorString(e));
  return 0;
}

int miclip_clock_probe(uint64_t* out, int32_t n_wg, void* stream) {
  if (!out || n_wg < 1 || n_wg > 4096) return fail(MICLIP_EINVAL, "bad argument to clock_probe");
  MICLIP_HIP(clock_probe((unsigned long long*)out, n_wg, (hipStream_t)stream));
  return 0;
}

int miclip_row_norms(const float* x, int32_t N, int32_t D, float* norms, float eps, float* out,
                     void* stream) {
  if (!x || !norms) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(row_norms(x, N, D, norms, (hipStream_t)stream));
  if (out) MICLIP_HIP(div_rows(x, norms, N, D, eps, out, (hipStream_t)stream));
  return 0;
}

int miclip_class_centroids(const float* x, const int32_t* order, const int32_t* offsets,
                           int32_t K, int32_t D, float eps, float* sums, float* centroids,
                           void* stream) {
  if (!x || !order || !offsets || !sums || !centroids) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(class_centroids(x, order, offsets, K, D, eps, sums, centroids, (hipStream_t)stream));
  return 0;
}

int miclip_proto_scores(const float* x, const float* protos, const int32_t* owner,
                        const int32_t* cls, const float* inv_nx, const float* inv_np, int32_t N,
                        int32_t P, int32_t D, float* own_best, int32_t* own_arg,
                        float* other_best, void* stream) {
  if (!x || !protos || !owner || !cls || !own_best || !own_arg || !other_best)
    return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(proto_scores(x, protos, owner, cls, inv_nx, inv_np, N, P, D, own_best, own_arg,
                          other_best, (hipStream_t)stream));
  return 0;
}

int miclip_set_profiling(miclip_model* m, int enable) {
  if (!m) return fail(MICLIP_EINVAL, "null model");
  m->profiling = enable != 0;
  return 0;
}

int miclip_profile_read(miclip_model* m, miclip_kernel_stat* out, int32_t n, int32_t reset) {
  if (!m) return fail(MICLIP_EINVAL, "null model");
  if ((int)m->prof_acc.size() < K_NUM) m->prof_acc.resize(K_NUM);
  for (auto& r : m->pending) {
    MICLIP_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    MICLIP_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    auto& acc = m->prof_acc[r.cls];
    acc.launches += 1;
    acc.ms += ms;
    acc.flops += r.flops;
    acc.bytes += r.bytes;
    m->event_pool.push_back(r.a);
    m->event_pool.push_back(r.b);
  }
  m->pending.clear();
  for (int i = 0; i < K_NUM && i < n && out; ++i) {
    out[i].name = kClassNames[i];
    out[i].launches = m->prof_acc[i].launches;
    out[i].ms = m->prof_acc[i].ms;
    out[i].flops = m->prof_acc[i].flops;
    out[i].bytes = m->prof_acc[i].bytes;
  }
  if (reset) m->prof_acc.assign(K_NUM, miclip_model::ProfAcc{});
  return K_NUM;
}

void miclip_model_destroy(miclip_model* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  for (auto& r : m->pending) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (hipEvent_t e : m->event_pool) (void)hipEventDestroy(e);
  if (m->ev_fork) (void)hipEventDestroy(m->ev_fork);
  for (int i = 0; i < 3; ++i) {
    if (m->ev_join[i]) (void)hipEventDestroy(m->ev_join[i]);
    if (m->aux[i]) (void)hipStreamDestroy(m->aux[i]);
  }
  pre_cache_destroy(m->pre);
  for (auto& kv : m->allocs) (void)hipFree(kv.first);
  delete m;
}

int64_t miclip_model_bytes(const miclip_model* m) { return m ? m->bytes : 0; }

int miclip_model_flags(const miclip_model* m) {
  if (!m) return 0;
  // ensure_folded skips the MX vision tower: LNFOLD names the vision tower only
  return (m->resid16 ? MICLIP_MODEL_RESID16 : 0) |
         (m->lnfold && !m->mx ? MICLIP_MODEL_LNFOLD : 0) |
         (m->lnfold ? MICLIP_MODEL_LNFOLD_TEXT : 0) |
         (m->mx ? MICLIP_MODEL_MXFP8 : 0) | (m->cls_last ? MICLIP_MODEL_CLS_LAST : 0) |
         (m->mx_out ? MICLIP_MODEL_MX_OUT : 0) |
         (m->mx && !m->mx_gelu_erf ? MICLIP_MODEL_MX_GELU_TANH : 0);
}

int miclip_set_gemm_variant(miclip_model* m, int32_t which, int32_t variant) {
  if (!m || which < 0 || which > 2) return fail(MICLIP_EINVAL, "bad argument to set_gemm_variant");
  if (which == 2) {   // MX-fp8 GEMMs: 0 default, 1 one tile per workgroup, 2 persistent
    if (variant < 0 || variant > 2)
      return fail(MICLIP_EINVAL, "MX gemm variant must be 0, 1 or 2 (bit-identical kernels)");
    m->gemm_variant[2] = variant;
    return 0;
  }
  if (variant != 0 && variant != 259)
    return fail(MICLIP_EINVAL, "gemm variant must be 0 or 259");
  m->gemm_variant[which] = variant;
  return 0;
}

int miclip_model_set_option(miclip_model* m, uint32_t option, int32_t on) {
  if (!m) return fail(MICLIP_EINVAL, "null model");
  if (option != MICLIP_OPT_FULL_LAST_BLOCK)
    return fail(MICLIP_EINVAL, "only MICLIP_OPT_FULL_LAST_BLOCK can change after create");
  m->cls_last = !on;
  return 0;
}

int miclip_op_gemm(int32_t dtype, const void* A, const void* W, const float* bias, void* C,
                   int32_t M, int32_t N, int32_t K, int32_t epi, int32_t act, int32_t variant,
                   void* stream) {
  if (!A || !W || !C) return fail(MICLIP_EINVAL, "null argument");
  hipStream_t s = (hipStream_t)stream;
  if (epi == 0) {
    MICLIP_HIP(gemm_store(dtype, A, W, bias, C, M, N, K, act, s, variant));
  } else if (epi == 1) {
    if (!bias) return fail(MICLIP_EINVAL, "residual epilogue needs a bias");
    MICLIP_HIP(gemm_residual(dtype, A, W, bias, (float*)C, M, N, K, s, variant));
  } else if (epi == 2) {
    MICLIP_HIP(gemm_f32(dtype, A, W, bias, (float*)C, M, N, K, s, variant));
  } else if (epi == 3) {
    MICLIP_HIP(gemm_null(dtype, A, W, (float*)C, M, N, K, s, variant));
  } else if (epi == 4) {
    if (!bias) return fail(MICLIP_EINVAL, "residual epilogue needs a bias");
    MICLIP_HIP(gemm_residual(dtype, A, W, bias, C, M, N, K, s, variant, 1));
  } else {
    return fail(MICLIP_EINVAL, "unknown epilogue");
  }
  return 0;
}

int miclip_op_gemm_splitk(int32_t dtype, const void* A, const void* W, const float* bias,
                          const float* c, const float* colsum, const float* stats, void* C,
                          int32_t M, int32_t N, int32_t K, int32_t epi, int32_t act, int32_t sk,
                          float* ws, void* stream) {
  if (!A || !W || !C || !ws) return fail(MICLIP_EINVAL, "null argument");
  if (sk < 2 || sk > 64) return fail(MICLIP_EINVAL, "sk must be in 2..64");
  hipStream_t s = (hipStream_t)stream;
  if (epi == 0) {
    MICLIP_HIP(gemm_store(dtype, A, W, bias, C, M, N, K, act, s, 0, ws, sk));
  } else if (epi == 1 || epi == 4) {
    if (!bias) return fail(MICLIP_EINVAL, "residual epilogue needs a bias");
    MICLIP_HIP(gemm_residual(dtype, A, W, bias, C, M, N, K, s, 0, epi == 4, ws, sk));
  } else if (epi == 5) {
    if (!c || !colsum || !stats) return fail(MICLIP_EINVAL, "folded-LN epilogue needs c, colsum, stats");
    MICLIP_HIP(gemm_store_ln(dtype, A, W, c, colsum, stats, C, M, N, K, act, s, 0, ws, sk));
  } else {
    return fail(MICLIP_EINVAL, "unknown epilogue");
  }
  return 0;
}

int miclip_op_ln_stats(const void* x, float* stats, int32_t R, int32_t D, const float* rscale,
                       void* stream) {
  if (!x || !stats) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(ln_stats(x, stats, R, D, (hipStream_t)stream, rscale));
  return 0;
}

int miclip_op_ln_fold(int32_t dtype, const void* W, const float* gamma, const float* beta,
                      const float* bias, void* Wf, float* colsum, float* c, int32_t N, int32_t K,
                      float* inv_scale, void* stream) {
  if (!W || !gamma || !beta || !Wf || !colsum || !c) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(ln_fold(dtype, W, gamma, beta, bias, Wf, colsum, c, N, K, (hipStream_t)stream,
                     inv_scale));
  return 0;
}

int miclip_op_gemm_ln(int32_t dtype, const void* A, const void* Wf, const float* c,
                      const float* colsum, const float* stats, void* C, int32_t M, int32_t N,
                      int32_t K, int32_t act, int32_t variant, void* stream) {
  if (!A || !Wf || !c || !colsum || !stats || !C) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(gemm_store_ln(dtype, A, Wf, c, colsum, stats, C, M, N, K, act, (hipStream_t)stream,
                           variant));
  return 0;
}

int miclip_op_layernorm(int32_t dtype, const void* in, const float* gamma, const float* beta,
                        void* out, int32_t flags, int32_t R, int32_t D, void* stream) {
  if (!in || !gamma || !beta || !out) return fail(MICLIP_EINVAL, "null argument");
  const bool of32 = flags & 1;
  MICLIP_HIP(layernorm(dtype, in, nullptr, 1, gamma, beta, of32 ? (float*)out : nullptr,
                       of32 ? nullptr : out, R, D, 0, (hipStream_t)stream, (flags >> 1) & 1));
  return 0;
}

int miclip_op_attention(int32_t dtype, const void* qkv, void* out, int32_t B, int32_t N,
                        int32_t H, int32_t head_dim, int32_t causal, int32_t variant,
                        void* stream) {
  if (!qkv || !out) return fail(MICLIP_EINVAL, "null argument");
  if (head_dim == 0) head_dim = 64;
  if (head_dim != 64 && head_dim != 80) return fail(MICLIP_EINVAL, "head_dim must be 64 or 80");
  MICLIP_HIP(attention(dtype, qkv, out, B, N, H, causal, (hipStream_t)stream, variant, head_dim));
  return 0;
}

int miclip_op_im2col(int32_t dtype, int32_t image_dtype, const void* images, void* patches,
                     int32_t B, int32_t R, int32_t P, int32_t Kp, int32_t variant, void* stream) {
  if (!images || !patches) return fail(MICLIP_EINVAL, "null argument");
  if (dtype != MICLIP_FP16 && dtype != MICLIP_BF16) return fail(MICLIP_EINVAL, "bad dtype");
  if (image_dtype != MICLIP_F32 && image_dtype != MICLIP_FP16 && image_dtype != MICLIP_BF16)
    return fail(MICLIP_EINVAL, "bad image dtype");
  const int in_dt = image_dtype == MICLIP_F32 ? kIn32 : image_dtype == MICLIP_FP16 ? kF16 : kBF16;
  MICLIP_HIP(im2col(dtype == MICLIP_FP16 ? kF16 : kBF16, in_dt, images, patches, B, R, P, Kp,
                    (hipStream_t)stream, variant));
  return 0;
}

int64_t miclip_mx_scale_bytes(int32_t rows, int32_t K) {
  return rows < 1 || K < 128 ? 0 : (int64_t)mx_scale_bytes(rows, K);
}

int miclip_op_attention_q0(int32_t dtype, const void* qkv, void* out, int32_t B, int32_t N,
                           int32_t H, int32_t head_dim, void* stream) {
  if (!qkv || !out) return fail(MICLIP_EINVAL, "null pointer");
  if (dtype != MICLIP_FP16 && dtype != MICLIP_BF16) return fail(MICLIP_EINVAL, "bad dtype");
  MICLIP_HIP(attention_q0(dtype, qkv, out, B, N, H, (hipStream_t)stream, head_dim));
  return 0;
}

int miclip_op_quant_mx(const void* in, int32_t in_f16, int32_t R, int32_t K, void* q, void* scales,
                       void* stream) {
  if (!in || !q || !scales) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(quant_mx(in_f16, in, R, K, q, scales, (hipStream_t)stream));
  return 0;
}

int miclip_op_gemm_mx(const void* A, const void* SA, const void* W, const void* SW,
                      const float* bias, void* C, void* CS, int32_t M, int32_t N, int32_t K,
                      int32_t epi, int32_t act, void* stream) {
  if (!A || !SA || !W || !SW || !C) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(gemm_mx(A, SA, W, SW, bias, C, CS, M, N, K, epi, act, (hipStream_t)stream));
  return 0;
}

int miclip_op_gemm_mx_v(const void* A, const void* SA, const void* W, const void* SW,
                        const float* bias, void* C, void* CS, int32_t M, int32_t N, int32_t K,
                        int32_t epi, int32_t act, int32_t variant, void* stream) {
  if (!A || !SA || !W || !SW || !C) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(gemm_mx(A, SA, W, SW, bias, C, CS, M, N, K, epi, act, (hipStream_t)stream, variant));
  return 0;
}

int miclip_op_layernorm_mx(const void* in, int32_t in_f16, const float* gamma, const float* beta,
                           void* q, void* scales, int32_t R, int32_t D, void* stream) {
  if (!in || !gamma || !beta || !q || !scales) return fail(MICLIP_EINVAL, "null argument");
  MICLIP_HIP(layernorm(MICLIP_FP16, in, nullptr, 1, gamma, beta, nullptr, nullptr, R, D, 0,
                       (hipStream_t)stream, in_f16, q, scales));
  return 0;
}

}  // extern "C"
