// Python bindings for the gfx950 kernels (torch tensors in, HIP launches on the
// current torch HIP stream out). Every entry point validates device, dtype,
// contiguity and shape on the host BEFORE launching, so a bad call raises a
// Python error instead of faulting the GPU.
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace caamd {
typedef __bf16 bf16;
void ln_fwd_launch(const bf16*, const bf16*, bf16*, const bf16*, const bf16*, bf16*, float*, float*,
                   int, int, float, hipStream_t);
void ln_bwd_launch(const bf16*, const bf16*, const bf16*, const float*, const float*, const bf16*,
                   bf16*, float*, bf16*, bf16*, int, int, hipStream_t, bf16*, int);
bool ln_bwd_dxsum_ok(int D);
int ln_nv_for(int D);
int ln_bwd_num_blocks(int rows);
int ln_bwd_partial_rows(int rows, int D);
void ln_bwd_config(int variant, int max_blocks);
void bias_gelu_fwd_launch(const bf16*, const bf16*, bf16*, int64_t, int, hipStream_t);
void bias_gelu_bwd_launch(const bf16*, const bf16*, const bf16*, bf16*, float*, bf16*, int, int,
                          hipStream_t);
int bias_gelu_bwd_slabs(int rows);
void xent_fwd_launch(const bf16*, const int64_t*, float*, float*, int, int, int, hipStream_t);
void xent_bwd_launch(bf16*, const int64_t*, const float*, const float*, int, int, int, hipStream_t);
hipError_t conv2d_launch(const bf16* X, const bf16* Wt, const bf16* bias, const bf16* R, bf16* Y, const bf16* zero,
                         int N, int H, int W, int lcin, int Ho, int Wo, int KH, int KW, int stride_h, int stride_w,
                         int pad_h, int pad_w, int Cout, int Kp, bool relu, int tile, hipStream_t st);
void normalize_pairs_launch(const uint8_t* in, bf16* out, int N, int H, int W, const float* sc, const float* bi,
                            hipStream_t st);
void normalize_pad8_launch(const uint8_t* in, bf16* out, int64_t npix, const float* sc, const float* bi,
                           hipStream_t st);
void maxpool3s2_launch(const bf16* x, bf16* y, int N, int H, int W, int C, int Ho, int Wo, hipStream_t st);
bool xent_fused_launch(bf16*, const int64_t*, float*, float*, const float*, int, int, int, hipStream_t);
void grad_sumsq_launch(const void*, bool, int64_t, float*, hipStream_t);
void adamw_config(int variant);
void fa64_set_pair(int v);
void adamw_launch(float*, float*, float*, const void*, bool, bf16*, int64_t, float, float, float,
                  float, float, float, float, float, float, const float*, const uint8_t*,
                  hipStream_t);
void gae_launch(const float*, const float*, const float*, float*, float*, int, int, float, float,
                hipStream_t);
void vtrace_launch(const float*, const float*, const float*, const float*, const float*, float*,
                   float*, int, int, float, float, hipStream_t);
hipError_t gemm_launch(int layout, int epi, int bm, int bn, const bf16* A, const bf16* B, void* C,
                       const bf16* bias, const bf16* Z, bf16* Zout, float* dbias, int M, int N,
                       int K, int lda, int ldb, int ldc, int splitk, int algo, hipStream_t st,
                       int tfull, int tS, float* tws, int* tcnt, int bpack);
void gemm_tail_plan(int tiles, int K, int ks, int slots, int max_split, int* full, int* S);
void gemm_set_tail_first(int v);
void gemm_set_group_m(int g);
void gemm_set_tn_group_m(int g);
hipError_t gemm_tn64_launch(int bm, bool accumulate, const bf16* A, const bf16* B, bf16* C, int M, int N, int K,
                            int lda, int ldb, int ldc, int slices, float* ws, hipStream_t st, int* tickets);
hipError_t gemm_nn64_launch(const bf16* A, const bf16* B, bf16* C, const bf16* bias, int M, int N, int K, int lda,
                            int ldb, int ldc, hipStream_t st);
void gemm_splitk_reduce(const float* part, int S, long long slab, bf16* out, int M, int N, int ldc,
                        bool accumulate, hipStream_t st);
void transpose_bf16(const bf16* in, bf16* out, int R, int C, hipStream_t st);
void decode_gemm_config(int ext);
hipError_t decode_gemm_norm_launch(const bf16* X, const bf16* W, float* part, int M, int N, int K, int ldx,
                                   int splits, bf16* res, const bf16* nw, bf16* h, float eps, hipStream_t st);
hipError_t decode_gemm_qkv_rope_launch(const bf16* X, const bf16* W, bf16* Y, float* part, int M, int N, int K,
                                       int ldx, int ldy, int splits, const float* cs, const int* pos,
                                       const int* slot, bf16* kc, bf16* vc, int H, int KVH, int BS,
                                       float* ssp, float eps, hipStream_t st);
hipError_t decode_gemm_launch(int epi, const bf16* X, const bf16* W, bf16* Y, const bf16* R, float* part,
                              unsigned* tick, int M, int N, int K, int ldx, int ldy, int splits, bool packed,
                              float* ssp, float eps, hipStream_t st);
void rl_gemm(int layout, const bf16* A, const bf16* B, void* C, const bf16* bias, const bf16* aux, int M, int N,
             int K, int lda, int ldb, int ldc, int epi, int splits, hipStream_t st);
void rl_im2col(const void* x, bool u8, bf16* col, int B, int H, int W, int C, int KH, int KW, int S, float scale,
               hipStream_t st);
void rl_col2im(const bf16* dcol, const bf16* y, bf16* dz, int B, int H, int W, int C, int KH, int KW, int S, int act,
               hipStream_t st);
void rl_colsum(const bf16* x, float* db, int M, int N, hipStream_t st);
void ppo_loss_cat(const float* logits, const float* vf, const int64_t* act, const float* old_logp,
                  const float* adv, const float* vt, const float* old_logits, int B, int A, float clip,
                  float vf_clip, float vf_coeff, float ent_coeff, float kl_coeff, const float* kl_dev,
                  float* dlogits, float* dvf, float* stats, hipStream_t st);
}  // namespace caamd

using at::Tensor;

#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype")
#define CHECK_BF16(t)          \
  do {                         \
    CHECK_GPU(t);              \
    CHECK_CONTIG(t);           \
    CHECK_DT(t, at::kBFloat16); \
  } while (0)
#define CHECK_F32(t)       \
  do {                     \
    CHECK_GPU(t);          \
    CHECK_CONTIG(t);       \
    CHECK_DT(t, at::kFloat); \
  } while (0)

// Every launch is followed by a check so a rejected launch (bad LDS size,
// bad grid) raises instead of leaving outputs silently unwritten.
#define LAUNCH_CHECK()                                                              \
  do {                                                                              \
    hipError_t e_ = hipGetLastError();                                              \
    TORCH_CHECK(e_ == hipSuccess, "HIP kernel launch failed: ", hipGetErrorString(e_)); \
  } while (0)

static inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
static inline caamd::bf16* bp(const Tensor& t) { return reinterpret_cast<caamd::bf16*>(t.data_ptr()); }
static inline caamd::bf16* bp_opt(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? bp(*t) : nullptr;
}

// ---- LayerNorm -------------------------------------------------------------
// returns (y, mean, rstd, s) where s = x + res when res is given (else undefined)
std::vector<Tensor> layernorm_fwd(const Tensor& x, const c10::optional<Tensor>& res,
                                  const Tensor& g, const Tensor& b, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(g);
  CHECK_BF16(b);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0, "layernorm: D must be a multiple of 8");
  TORCH_CHECK(caamd::ln_nv_for(D) > 0, "layernorm: D too large (max 4096)");
  TORCH_CHECK(g.numel() == D && b.numel() == D, "layernorm: weight/bias size mismatch");
  const int rows = (int)(x.numel() / D);
  Tensor s;
  if (res.has_value() && res->defined()) {
    CHECK_BF16(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "layernorm: residual shape mismatch");
    s = at::empty_like(x);
  }
  auto y = at::empty_like(x);
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  if (rows > 0)
    caamd::ln_fwd_launch(bp(x), bp_opt(res), s.defined() ? bp(s) : nullptr, bp(g), bp(b), bp(y),
                         mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, D, (float)eps,
                         cur_stream());
    LAUNCH_CHECK();
  return {y, mean, rstd, s};
}

// returns (dx, dg, db); dx += dres when dres given
// dxsum (optional bf16 [D], only where ln_bwd_dxsum_ok(D)): += column sums of dx,
// i.e. the bias gradient of the layer that produced the residual branch.
std::vector<Tensor> layernorm_bwd(const Tensor& dy, const Tensor& x, const Tensor& g,
                                  const Tensor& mean, const Tensor& rstd,
                                  const c10::optional<Tensor>& dres,
                                  const c10::optional<Tensor>& dxsum,
                                  const c10::optional<Tensor>& g_main,
                                  const c10::optional<Tensor>& b_main) {
  CHECK_BF16(dy);
  CHECK_BF16(x);
  CHECK_BF16(g);
  CHECK_F32(mean);
  CHECK_F32(rstd);
  TORCH_CHECK(dy.sizes() == x.sizes(), "layernorm_bwd: dy/x shape mismatch");
  const int D = (int)x.size(-1);
  const int rows = (int)(x.numel() / D);
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_bwd: stats size");
  if (dres.has_value() && dres->defined()) {
    CHECK_BF16(*dres);
    TORCH_CHECK(dres->sizes() == x.sizes(), "layernorm_bwd: dres shape mismatch");
  }
  auto dx = at::empty_like(x);
  // g_main / b_main: the LayerNorm's own main-grad views; the column sums are added into
  // them in the same launch and dg / db come back undefined (None)
  const bool acc = g_main.has_value() && g_main->defined();
  TORCH_CHECK(acc == (b_main.has_value() && b_main->defined()), "layernorm_bwd: g_main and b_main go together");
  Tensor dg, db;
  if (acc) {
    for (const Tensor* t : {&*g_main, &*b_main}) {
      CHECK_BF16(*t);
      TORCH_CHECK(t->numel() == D && t->is_contiguous() && t->device() == x.device(),
                  "layernorm_bwd: main grads must be contiguous [D] on the input's device");
    }
    dg = *g_main;
    db = *b_main;
  } else {
    dg = at::empty_like(g);
    db = at::empty_like(g);
  }
  caamd::bf16* dxs = nullptr;
  if (dxsum.has_value() && dxsum->defined()) {
    CHECK_BF16(*dxsum);
    TORCH_CHECK(dxsum->numel() == D && caamd::ln_bwd_dxsum_ok(D), "layernorm_bwd: dxsum needs [D] and the cs path");
    dxs = bp(*dxsum);
  }
  const int nblk = caamd::ln_bwd_partial_rows(rows, D);
  auto partial = at::empty({nblk, dxs ? 3 : 2, D}, x.options().dtype(at::kFloat));
  if (rows > 0) {
    caamd::ln_bwd_launch(bp(dy), bp(x), bp(g), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                         bp_opt(dres), bp(dx), partial.data_ptr<float>(), bp(dg), bp(db), rows, D,
                         cur_stream(), dxs, acc ? 1 : 0);
    LAUNCH_CHECK();
  } else if (!acc) {
    dg.zero_();
    db.zero_();
  }
  if (acc) return {dx, Tensor(), Tensor()};
  return {dx, dg, db};
}

// ---- bias + GELU -------------------------------------------------------------
Tensor bias_gelu_fwd(const Tensor& h, const c10::optional<Tensor>& b) {
  CHECK_BF16(h);
  const int N = (int)h.size(-1);
  TORCH_CHECK(N % 8 == 0, "bias_gelu: last dim must be a multiple of 8");
  if (b.has_value() && b->defined()) {
    CHECK_BF16(*b);
    TORCH_CHECK(b->numel() == N, "bias_gelu: bias size mismatch");
  }
  auto y = at::empty_like(h);
  const int64_t rows = h.numel() / N;
  if (rows > 0) caamd::bias_gelu_fwd_launch(bp(h), bp_opt(b), bp(y), rows, N, cur_stream());
  LAUNCH_CHECK();
  return y;
}

std::vector<Tensor> bias_gelu_bwd(const Tensor& dy, const Tensor& h,
                                  const c10::optional<Tensor>& b) {
  CHECK_BF16(dy);
  CHECK_BF16(h);
  TORCH_CHECK(dy.sizes() == h.sizes(), "bias_gelu_bwd: shape mismatch");
  const int N = (int)h.size(-1);
  TORCH_CHECK(N % 8 == 0, "bias_gelu_bwd: last dim must be a multiple of 8");
  const int64_t rows64 = h.numel() / N;
  TORCH_CHECK(rows64 < (1ll << 31), "bias_gelu_bwd: too many rows");
  const int rows = (int)rows64;
  const bool has_b = b.has_value() && b->defined();
  if (has_b) CHECK_BF16(*b);
  auto dh = at::empty_like(h);
  Tensor db, partial;
  if (has_b) {
    db = at::empty_like(*b);
    partial = at::empty({caamd::bias_gelu_bwd_slabs(rows), N}, h.options().dtype(at::kFloat));
  }
  if (rows > 0)
    caamd::bias_gelu_bwd_launch(bp(dy), bp(h), bp_opt(b), bp(dh),
                                has_b ? partial.data_ptr<float>() : nullptr,
                                has_b ? bp(db) : nullptr, rows, N, cur_stream());
    LAUNCH_CHECK();
  return {dh, db};
}

// ---- bias gradient (column sum of dy), optionally accumulated in place -----------
namespace caamd {
void bias_grad_launch(const bf16*, float*, bf16*, int, int, int, hipStream_t);
void drain_f32_launch(float*, bf16*, int, hipStream_t);
}

// dst (bf16) += src (fp32); src = 0 (an fp32 bias-gradient accumulator drained into a
// main gradient, ready for its next use)
void drain_f32_(Tensor& src, Tensor& dst) {
  CHECK_F32(src);
  CHECK_BF16(dst);
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && src.numel() == dst.numel() &&
                  src.device() == dst.device(),
              "drain_f32_: contiguous src/dst of equal size on one device");
  if (src.numel() > 0) {
    caamd::drain_f32_launch(src.data_ptr<float>(), bp(dst), (int)src.numel(), cur_stream());
    LAUNCH_CHECK();
  }
}

void bias_grad_(const Tensor& dy2d, Tensor& out, bool accumulate) {
  CHECK_BF16(dy2d);
  CHECK_BF16(out);
  TORCH_CHECK(dy2d.dim() == 2, "bias_grad: dy must be 2-D");
  const int rows = (int)dy2d.size(0), N = (int)dy2d.size(1);
  TORCH_CHECK(N % 8 == 0, "bias_grad: N must be a multiple of 8");
  TORCH_CHECK(out.numel() == N, "bias_grad: out size mismatch");
  auto partial = at::empty({caamd::bias_gelu_bwd_slabs(rows), N}, dy2d.options().dtype(at::kFloat));
  if (rows > 0) {
    caamd::bias_grad_launch(bp(dy2d), partial.data_ptr<float>(), bp(out), rows, N, accumulate ? 1 : 0,
                            cur_stream());
    LAUNCH_CHECK();
  } else if (!accumulate) {
    out.zero_();
  }
}

// ---- cross entropy -----------------------------------------------------------
// logits [N, stride] bf16 (columns >= V are padding), target [N] int64.
std::vector<Tensor> xent_fwd(const Tensor& logits, const Tensor& target, int64_t V) {
  CHECK_BF16(logits);
  CHECK_GPU(target);
  CHECK_CONTIG(target);
  CHECK_DT(target, at::kLong);
  TORCH_CHECK(logits.dim() == 2, "xent: logits must be 2-D");
  const int rows = (int)logits.size(0), stride = (int)logits.size(1);
  TORCH_CHECK(stride % 8 == 0, "xent: row stride must be a multiple of 8");
  TORCH_CHECK(V > 0 && V <= stride, "xent: bad vocab size");
  TORCH_CHECK(target.numel() == rows, "xent: target size mismatch");
  auto loss = at::empty({rows}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({rows}, logits.options().dtype(at::kFloat));
  if (rows > 0)
    caamd::xent_fwd_launch(bp(logits), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                           lse.data_ptr<float>(), rows, (int)V, stride, cur_stream());
    LAUNCH_CHECK();
  return {loss, lse};
}

// In place: logits <- dlogits.
void xent_bwd_(Tensor& logits, const Tensor& target, const Tensor& lse, const Tensor& dl,
               int64_t V) {
  CHECK_BF16(logits);
  CHECK_F32(lse);
  CHECK_F32(dl);
  CHECK_DT(target, at::kLong);
  const int rows = (int)logits.size(0), stride = (int)logits.size(1);
  TORCH_CHECK(stride % 8 == 0 && V <= stride, "xent_bwd: bad stride/V");
  TORCH_CHECK(target.numel() == rows && lse.numel() == rows && dl.numel() == rows,
              "xent_bwd: size mismatch");
  if (rows > 0)
    caamd::xent_bwd_launch(bp(logits), target.data_ptr<int64_t>(), lse.data_ptr<float>(),
                           dl.data_ptr<float>(), rows, (int)V, stride, cur_stream());
    LAUNCH_CHECK();
}

// Fused forward + backward, in place: logits <- scale * (softmax - onehot); returns
// {loss, lse} per row. scale: 1-element fp32 device tensor (no host sync).
std::vector<Tensor> xent_fused_(Tensor& logits, const Tensor& target, const Tensor& scale, int64_t V) {
  CHECK_BF16(logits);
  CHECK_GPU(target);
  CHECK_CONTIG(target);
  CHECK_DT(target, at::kLong);
  CHECK_F32(scale);
  TORCH_CHECK(logits.dim() == 2, "xent_fused: logits must be 2-D");
  const int rows = (int)logits.size(0), stride = (int)logits.size(1);
  TORCH_CHECK(stride % 8 == 0 && V > 0 && V <= stride, "xent_fused: bad stride/V");
  TORCH_CHECK(target.numel() == rows && scale.numel() == 1, "xent_fused: size mismatch");
  TORCH_CHECK(((uintptr_t)logits.data_ptr()) % 16 == 0, "xent_fused: 16-byte alignment");
  auto loss = at::empty({rows}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({rows}, logits.options().dtype(at::kFloat));
  if (rows > 0) {
    TORCH_CHECK(caamd::xent_fused_launch(bp(logits), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                         lse.data_ptr<float>(), scale.data_ptr<float>(), rows, (int)V, stride,
                                         cur_stream()),
                "xent_fused: row too wide for the register-resident kernel");
    LAUNCH_CHECK();
  }
  return {loss, lse};
}

// ---- optimizer ---------------------------------------------------------------
void grad_sumsq(const Tensor& g, Tensor& out) {
  CHECK_GPU(g);
  CHECK_CONTIG(g);
  CHECK_F32(out);
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat,
              "grad_sumsq: grad must be bf16 or fp32");
  TORCH_CHECK(g.numel() % 8 == 0, "grad_sumsq: numel must be a multiple of 8");
  if (g.numel() > 0)
    caamd::grad_sumsq_launch(g.data_ptr(), g.scalar_type() == at::kBFloat16, g.numel(),
                             out.data_ptr<float>(), cur_stream());
    LAUNCH_CHECK();
}

void adamw_step(Tensor& p, Tensor& m, Tensor& v, const Tensor& g,
                const c10::optional<Tensor>& pbf, double lr, double beta1, double beta2,
                double eps, double wd, int64_t step, double inv_world, double max_norm,
                const c10::optional<Tensor>& sumsq, const c10::optional<Tensor>& wd_mask) {
  CHECK_F32(p);
  CHECK_F32(m);
  CHECK_F32(v);
  CHECK_GPU(g);
  CHECK_CONTIG(g);
  const int64_t n = p.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n, "adamw: size mismatch");
  TORCH_CHECK(n % 8 == 0, "adamw: numel must be a multiple of 8 (pad the flat buffer)");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat,
              "adamw: grad must be bf16 or fp32");
  if (pbf.has_value() && pbf->defined()) {
    CHECK_BF16(*pbf);
    TORCH_CHECK(pbf->numel() == n, "adamw: bf16 copy size mismatch");
  }
  const float* ss = nullptr;
  if (sumsq.has_value() && sumsq->defined()) {
    CHECK_F32(*sumsq);
    ss = sumsq->data_ptr<float>();
  }
  const uint8_t* mask = nullptr;
  if (wd_mask.has_value() && wd_mask->defined()) {
    CHECK_GPU(*wd_mask);
    CHECK_CONTIG(*wd_mask);
    CHECK_DT(*wd_mask, at::kByte);
    TORCH_CHECK(wd_mask->numel() == n / 8, "adamw: wd_mask must have numel/8 entries");
    mask = wd_mask->data_ptr<uint8_t>();
  }
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  if (n > 0)
    caamd::adamw_launch(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                        g.data_ptr(), g.scalar_type() == at::kBFloat16, bp_opt(pbf), n, (float)lr,
                        (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                        (float)inv_world, (float)max_norm, ss, mask, cur_stream());
    LAUNCH_CHECK();
}

// ---- RL returns (time-major [T, B], fp32) ----------------------------------------
std::vector<Tensor> gae(const Tensor& rewards, const Tensor& values, const Tensor& nonterminal,
                        double gamma, double lam) {
  CHECK_F32(rewards);
  CHECK_F32(values);
  CHECK_F32(nonterminal);
  TORCH_CHECK(rewards.dim() == 2, "gae: rewards must be [T, B]");
  const int T = (int)rewards.size(0), B = (int)rewards.size(1);
  TORCH_CHECK(values.dim() == 2 && values.size(0) == T + 1 && values.size(1) == B,
              "gae: values must be [T+1, B]");
  TORCH_CHECK(nonterminal.sizes() == rewards.sizes(), "gae: nonterminal must be [T, B]");
  auto adv = at::empty_like(rewards), tgt = at::empty_like(rewards);
  if (T > 0 && B > 0)
    caamd::gae_launch(rewards.data_ptr<float>(), values.data_ptr<float>(),
                      nonterminal.data_ptr<float>(), adv.data_ptr<float>(), tgt.data_ptr<float>(),
                      T, B, (float)gamma, (float)lam, cur_stream());
    LAUNCH_CHECK();
  return {adv, tgt};
}

std::vector<Tensor> vtrace(const Tensor& log_rhos, const Tensor& discounts, const Tensor& rewards,
                           const Tensor& values, const Tensor& bootstrap, double clip_rho,
                           double clip_pg_rho) {
  CHECK_F32(log_rhos);
  CHECK_F32(discounts);
  CHECK_F32(rewards);
  CHECK_F32(values);
  CHECK_F32(bootstrap);
  TORCH_CHECK(log_rhos.dim() == 2, "vtrace: inputs must be [T, B]");
  const int T = (int)log_rhos.size(0), B = (int)log_rhos.size(1);
  TORCH_CHECK(discounts.sizes() == log_rhos.sizes() && rewards.sizes() == log_rhos.sizes() &&
                  values.sizes() == log_rhos.sizes(),
              "vtrace: shape mismatch");
  TORCH_CHECK(bootstrap.numel() == B, "vtrace: bootstrap must be [B]");
  auto vs = at::empty_like(values), pg = at::empty_like(values);
  if (T > 0 && B > 0)
    caamd::vtrace_launch(log_rhos.data_ptr<float>(), discounts.data_ptr<float>(),
                         rewards.data_ptr<float>(), values.data_ptr<float>(),
                         bootstrap.data_ptr<float>(), vs.data_ptr<float>(), pg.data_ptr<float>(),
                         T, B, (float)clip_rho, (float)clip_pg_rho, cur_stream());
    LAUNCH_CHECK();
  return {vs, pg};
}

// ---- flash attention (packed qkv [B, T, 3*H*D]) ---------------------------------
namespace caamd {
void fa_fwd_launch(const bf16*, bf16*, float*, int, int, int, int, int, hipStream_t);
bool fa_bwd_launch(const bf16* qkv, const bf16* out, const bf16* dout, const float* lse, float* delta, bf16* dqkv,
                   int B, int T, int H, int D, int causal, hipStream_t st, float* dbias);
}

static void fa_check_qkv(const Tensor& qkv, int64_t H, int& B, int& T, int& D) {
  CHECK_BF16(qkv);
  TORCH_CHECK(qkv.dim() == 3, "flash_attn: qkv must be [B, T, 3*H*D]");
  B = (int)qkv.size(0);
  T = (int)qkv.size(1);
  TORCH_CHECK(qkv.size(2) % (3 * H) == 0, "flash_attn: last dim must be 3*H*D");
  D = (int)(qkv.size(2) / (3 * H));
  TORCH_CHECK(D == 64 || D == 128, "flash_attn: head dim must be 64 or 128");
}

std::vector<Tensor> flash_attn_fwd(const Tensor& qkv, int64_t H, bool causal) {
  int B, T, D;
  fa_check_qkv(qkv, H, B, T, D);
  auto out = at::empty({B, T, H * D}, qkv.options());
  auto lse = at::empty({B, H, T}, qkv.options().dtype(at::kFloat));
  if (B > 0 && T > 0)
    caamd::fa_fwd_launch(bp(qkv), bp(out), lse.data_ptr<float>(), B, T, (int)H, D, causal ? 1 : 0,
                         cur_stream());
    LAUNCH_CHECK();
  return {out, lse};
}

// dbias (optional fp32 [3*H*D]): += column sums of dqkv over the tokens (the qkv
// projection's bias gradient), from the kernels' registers where they support it.
Tensor flash_attn_bwd(const Tensor& qkv, const Tensor& out, const Tensor& dout, const Tensor& lse,
                      int64_t H, bool causal, const c10::optional<Tensor>& dbias) {
  int B, T, D;
  fa_check_qkv(qkv, H, B, T, D);
  CHECK_BF16(out);
  CHECK_BF16(dout);
  CHECK_F32(lse);
  TORCH_CHECK(out.dim() == 3 && out.size(0) == B && out.size(1) == T && out.size(2) == H * D,
              "flash_attn_bwd: out shape");
  TORCH_CHECK(dout.sizes() == out.sizes(), "flash_attn_bwd: dout shape");
  TORCH_CHECK(lse.numel() == (int64_t)B * H * T, "flash_attn_bwd: lse shape");
  auto dqkv = at::empty_like(qkv);
  // workspace: Delta = rowsum(dO * O) and lse * log2(e), [2, B, H, T]
  auto delta = at::empty({2, (int64_t)B * H * T}, lse.options());
  float* dbp = nullptr;
  if (dbias.has_value()) {
    CHECK_F32(*dbias);
    TORCH_CHECK(dbias->numel() == 3 * H * D, "flash_attn_bwd: dbias must have 3*H*D elements");
    dbp = dbias->data_ptr<float>();
  }
  if (B > 0 && T > 0) {
    const bool done = caamd::fa_bwd_launch(bp(qkv), bp(out), bp(dout), lse.data_ptr<float>(),
                                           delta.data_ptr<float>(), bp(dqkv), B, T, (int)H, D, causal ? 1 : 0,
                                           cur_stream(), dbp);
    LAUNCH_CHECK();
    if (!done) {
      Tensor d = dbias.value();
      d.add_(dqkv.reshape({-1, 3 * H * D}).sum(0, false, at::kFloat));
    }
  }
  return dqkv;
}

// ---- LLM serving kernels (llm.hip) -------------------------------------------------
namespace caamd {
void rmsnorm_launch(const bf16*, const bf16*, bf16*, const bf16*, bf16*, int, int, float, hipStream_t);
void silu_mul_launch(const bf16*, bf16*, int, int, hipStream_t);
void argmax_rows_launch(const bf16* x, int M, int V, long long ld, long long* out, hipStream_t st);
void rope_cache_launch(bf16*, const float*, const int*, const int*, bf16*, bf16*, int, int, int, int, int,
                       hipStream_t);
bool paged_decode_launch(const bf16*, int, const bf16*, const bf16*, const int*, int, const int*, bf16*, float*,
                         float*, int, int, int, int, int, int, float, hipStream_t);
int paged_max_parts(int);
int paged_mfma_max_parts(int);
bool paged_decode_mfma_launch(const bf16*, int, const bf16*, const bf16*, const int*, int, const int*, bf16*,
                              float*, float*, int, int, int, int, int, int, float, hipStream_t);
void fa_fwd_gqa_launch(const bf16*, const bf16*, const bf16*, int, int, int, bf16*, float*, int, int, int, int,
                       int, hipStream_t);
}

std::vector<Tensor> rmsnorm(const Tensor& x, const Tensor& w, double eps, const c10::optional<Tensor>& residual) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 16 * 512, "rmsnorm: D must be a multiple of 8 and <= 8192");
  TORCH_CHECK(w.numel() == D, "rmsnorm: weight size");
  const int rows = (int)(x.numel() / D);
  auto y = at::empty_like(x);
  Tensor s_out;
  const caamd::bf16* r = nullptr;
  if (residual.has_value()) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->sizes() == x.sizes(), "rmsnorm: residual shape");
    s_out = at::empty_like(x);
    r = bp(*residual);
  }
  if (rows > 0) {
    caamd::rmsnorm_launch(bp(x), r, r ? bp(s_out) : nullptr, bp(w), bp(y), rows, D, (float)eps, cur_stream());
    LAUNCH_CHECK();
  }
  return {y, s_out};
}

// greedy sampling: argmax over the last dim of bf16 logits [M, V] -> int64 [M]
// (first maximum on ties)
Tensor argmax_rows(const Tensor& x) {
  CHECK_GPU(x);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) > 0, "argmax_rows: [M, V] with unit column stride");
  Tensor out = torch::empty({x.size(0)}, x.options().dtype(at::kLong));
  if (x.size(0) > 0)
    caamd::argmax_rows_launch((const caamd::bf16*)x.data_ptr(), (int)x.size(0), (int)x.size(1),
                              (long long)x.stride(0), (long long*)out.data_ptr<int64_t>(), cur_stream());
  return out;
}

Tensor silu_mul(const Tensor& gu) {
  CHECK_BF16(gu);
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "silu_mul: last dim must be 2*F with F % 8 == 0");
  const int F = (int)(F2 / 2);
  const int rows = (int)(gu.numel() / F2);
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto out = at::empty(sizes, gu.options());
  if (rows > 0) {
    caamd::silu_mul_launch(bp(gu), bp(out), rows, F, cur_stream());
    LAUNCH_CHECK();
  }
  return out;
}

void rope_cache_(Tensor& qkv, const Tensor& cos_sin, const Tensor& positions, const c10::optional<Tensor>& slots,
                 const c10::optional<Tensor>& k_cache, const c10::optional<Tensor>& v_cache, int64_t H,
                 int64_t KVH) {
  CHECK_BF16(qkv);
  CHECK_F32(cos_sin);
  CHECK_GPU(positions);
  CHECK_CONTIG(positions);
  CHECK_DT(positions, at::kInt);
  const int N = (int)positions.numel();
  TORCH_CHECK(qkv.numel() % ((int64_t)N * (H + 2 * KVH)) == 0, "rope_cache: qkv shape");
  const int D = (int)(qkv.numel() / ((int64_t)N * (H + 2 * KVH)));
  TORCH_CHECK(D % 16 == 0 && cos_sin.size(-2) == D / 2 && cos_sin.size(-1) == 2, "rope_cache: head dim must be a multiple of 16 and cos_sin [P, D/2, 2]");
  caamd::bf16 *kc = nullptr, *vc = nullptr;
  const int* sl = nullptr;
  int BS = 1;
  if (k_cache.has_value()) {
    TORCH_CHECK(slots.has_value() && v_cache.has_value(), "rope_cache: slots and v_cache required with k_cache");
    CHECK_BF16(*k_cache);
    CHECK_BF16(*v_cache);
    CHECK_DT(*slots, at::kInt);
    TORCH_CHECK(slots->numel() == N, "rope_cache: slots shape");
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == KVH && k_cache->size(3) == D,
                "rope_cache: cache must be [num_blocks, KVH, BS, D]");
    BS = (int)k_cache->size(2);
    kc = bp(*k_cache);
    vc = bp(*v_cache);
    sl = slots->data_ptr<int>();
  }
  if (N > 0) {
    caamd::rope_cache_launch(bp(qkv), cos_sin.data_ptr<float>(), positions.data_ptr<int>(), sl, kc, vc, N, (int)H,
                             (int)KVH, D, BS, cur_stream());
    LAUNCH_CHECK();
  }
}

// impl: -1 auto (MFMA kernel for D=128 / 16-token pages / G <= 16 unless CAAMD_PAGED_MFMA=0),
//        0 the VALU kernel, 1 the MFMA kernel
Tensor paged_decode(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                    const Tensor& ctx_lens, int64_t max_ctx, int64_t H, double scale, int64_t impl) {
  CHECK_GPU(q);
  CHECK_DT(q, at::kBFloat16);
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1, "paged_decode: q must be [B, >=H*D] with unit inner stride");
  CHECK_BF16(k_cache);
  CHECK_BF16(v_cache);
  TORCH_CHECK(k_cache.dim() == 4, "paged_decode: cache must be [num_blocks, KVH, BS, D]");
  const int KVH = (int)k_cache.size(1), BS = (int)k_cache.size(2), D = (int)k_cache.size(3);
  const int B = (int)q.size(0);
  TORCH_CHECK(q.size(1) >= H * D, "paged_decode: q width");
  TORCH_CHECK(H % KVH == 0, "paged_decode: H must be a multiple of KVH");
  CHECK_GPU(block_tables);
  CHECK_CONTIG(block_tables);
  CHECK_DT(block_tables, at::kInt);
  CHECK_GPU(ctx_lens);
  CHECK_DT(ctx_lens, at::kInt);
  TORCH_CHECK(block_tables.size(0) == B && ctx_lens.numel() == B, "paged_decode: batch mismatch");
  TORCH_CHECK(max_ctx <= block_tables.size(1) * BS, "paged_decode: max_ctx exceeds block table capacity");
  auto out = at::empty({B, H * D}, q.options());
  const int G = (int)(H / KVH);
  const bool mfma_ok = D == 128 && BS == 16 && (G == 1 || G == 2 || G == 4 || G == 8 || G == 16);
  if (impl < 0) {
    const char* e = std::getenv("CAAMD_PAGED_MFMA");
    impl = (mfma_ok && !(e && e[0] == '0')) ? 1 : 0;
  }
  TORCH_CHECK(impl == 0 || mfma_ok, "paged_decode: the MFMA kernel needs D=128, 16-token pages, H/KVH in {1..16}");
  const int mp = impl == 1 ? caamd::paged_mfma_max_parts((int)max_ctx) : caamd::paged_max_parts((int)max_ctx);
  Tensor pacc, pml;
  if (mp > 1) {
    pacc = at::empty({B, H, mp, D}, q.options().dtype(at::kFloat));
    pml = at::empty({B, H, mp, 2}, q.options().dtype(at::kFloat));
  }
  if (B > 0) {
    float* pa = mp > 1 ? pacc.data_ptr<float>() : nullptr;
    float* pm = mp > 1 ? pml.data_ptr<float>() : nullptr;
    const bool ok = impl == 1
        ? caamd::paged_decode_mfma_launch(bp(q), (int)q.stride(0), bp(k_cache), bp(v_cache),
                                          block_tables.data_ptr<int>(), (int)block_tables.size(1),
                                          ctx_lens.data_ptr<int>(), bp(out), pa, pm, B, (int)H, KVH, D, BS,
                                          (int)max_ctx, (float)scale, cur_stream())
        : caamd::paged_decode_launch(bp(q), (int)q.stride(0), bp(k_cache), bp(v_cache), block_tables.data_ptr<int>(),
                                     (int)block_tables.size(1), ctx_lens.data_ptr<int>(), bp(out), pa, pm, B, (int)H,
                                     KVH, D, BS, (int)max_ctx, (float)scale, cur_stream());
    TORCH_CHECK(ok, "paged_decode: unsupported head_dim/group (D in {64,128}, H/KVH in {1,2,4,8})");
    LAUNCH_CHECK();
  }
  return out;
}

// q/k/v: [B, T, width] views (e.g. slices of one fused qkv projection) with unit inner stride
std::vector<Tensor> flash_attn_gqa(const Tensor& q, const Tensor& k, const Tensor& v, int64_t H, int64_t KVH,
                                   bool causal) {
  for (const Tensor* t : {&q, &k, &v}) {
    CHECK_GPU(*t);
    CHECK_DT(*t, at::kBFloat16);
    TORCH_CHECK(t->dim() == 3 && t->stride(2) == 1 && t->stride(0) == t->size(1) * t->stride(1),
                "flash_attn_gqa: q/k/v must be [B, T, width] with dense rows");
  }
  const int B = (int)q.size(0), T = (int)q.size(1);
  TORCH_CHECK(q.size(2) % H == 0, "flash_attn_gqa: q width");
  const int D = (int)(q.size(2) / H);
  TORCH_CHECK(D == 64 || D == 128, "flash_attn_gqa: head dim must be 64 or 128");
  TORCH_CHECK(k.size(2) == KVH * D && v.size(2) == KVH * D && H % KVH == 0, "flash_attn_gqa: kv width");
  TORCH_CHECK(k.stride(1) == v.stride(1), "flash_attn_gqa: k/v row strides differ");
  auto out = at::empty({B, T, H * D}, q.options());
  auto lse = at::empty({B, H, T}, q.options().dtype(at::kFloat));
  if (B > 0 && T > 0) {
    caamd::fa_fwd_gqa_launch(bp(q), bp(k), bp(v), (int)q.stride(1), (int)k.stride(1), (int)(H / KVH), bp(out),
                             lse.data_ptr<float>(), B, T, (int)H, D, causal ? 1 : 0, cur_stream());
    LAUNCH_CHECK();
  }
  return {out, lse};
}

// ---- vision (Data GPU map_batches / ResNet-50) ------------------------------
namespace caamd {
void image_normalize_launch(const uint8_t*, bf16*, int64_t, const float*, const float*, hipStream_t);
void add_relu_launch(bf16*, const bf16*, int64_t, hipStream_t);
void bias_act_launch(bf16*, const bf16*, const bf16*, int64_t, int, bool, hipStream_t);
}

// y: [N, C, H, W] bf16 in channels_last (physically NHWC), b: [C]; in place.
void bias_act_(Tensor& y, const Tensor& b, const c10::optional<Tensor>& r, bool relu) {
  CHECK_GPU(y);
  CHECK_DT(y, at::kBFloat16);
  CHECK_BF16(b);
  TORCH_CHECK(y.dim() == 4 && y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bias_act_: y must be 4-D channels_last");
  const int C = (int)y.size(1);
  TORCH_CHECK(C % 8 == 0 && b.numel() == C, "bias_act_: C % 8 == 0 and bias of size C");
  const caamd::bf16* rp = nullptr;
  if (r.has_value()) {
    CHECK_GPU(*r);
    CHECK_DT(*r, at::kBFloat16);
    TORCH_CHECK(r->sizes() == y.sizes() && r->strides() == y.strides(), "bias_act_: residual layout");
    rp = bp(*r);
  }
  if (y.numel()) caamd::bias_act_launch(bp(y), bp(b), rp, y.numel(), C, relu, cur_stream());
  LAUNCH_CHECK();
}

Tensor image_normalize(const Tensor& x, std::vector<double> mean, std::vector<double> std) {
  CHECK_GPU(x);
  CHECK_CONTIG(x);
  CHECK_DT(x, at::kByte);
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3, "image_normalize: expects uint8 [N, H, W, 3]");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "image_normalize: 3 means / stds");
  TORCH_CHECK(((uintptr_t)x.data_ptr()) % 16 == 0, "image_normalize: input must be 16-byte aligned");
  // bf16 [N, 3, H, W] in channels_last = physically NHWC, the same element order as x
  auto out = at::empty({x.size(0), 3, x.size(1), x.size(2)},
                       x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
  float sc[3], bi[3];
  for (int c = 0; c < 3; ++c) {
    sc[c] = (float)(1.0 / (255.0 * std[c]));
    bi[c] = (float)(-mean[c] / std[c]);
  }
  if (x.numel())
    caamd::image_normalize_launch(x.data_ptr<uint8_t>(), bp(out), x.numel(), sc, bi, cur_stream());
  LAUNCH_CHECK();
  return out;
}

// ---- implicit-GEMM NHWC convolution (conv.hip) ----------------------------------
// x [N, H, W, Cin] (plain contiguous NHWC), w [Cout, Kp] with k = (kh*KS + kw)*Cin + ci
// (zero-padded to Kp % 32 == 0), bias [Cout]; residual [N, Ho, Wo, Cout] or None.
// y = act(conv(x, w) + bias (+ residual)); tile 0 = 256x128, 1 = 256x64, 2 = 128x128.
Tensor conv2d_nhwc_ex(const Tensor& x, const Tensor& w, const Tensor& bias, c10::optional<Tensor> residual,
                      int64_t kh, int64_t kw, int64_t stride, int64_t stride_w, int64_t pad, int64_t pad_w, bool relu,
                      int64_t tile, const Tensor& zero);

Tensor conv2d_nhwc(const Tensor& x, const Tensor& w, const Tensor& bias, c10::optional<Tensor> residual,
                   int64_t ks, int64_t stride, int64_t pad, bool relu, int64_t tile, const Tensor& zero) {
  return conv2d_nhwc_ex(x, w, bias, residual, ks, ks, stride, stride, pad, pad, relu, tile, zero);
}

// General form: kh x kw kernel (1x1, 3x3, 7x7, or the pixel-pair stem's 7x4), stride and
// padding per direction (stride / pad: vertical, stride_w / pad_w: horizontal).
Tensor conv2d_nhwc_ex(const Tensor& x, const Tensor& w, const Tensor& bias, c10::optional<Tensor> residual,
                      int64_t kh, int64_t kw, int64_t stride, int64_t stride_w, int64_t pad, int64_t pad_w, bool relu,
                      int64_t tile, const Tensor& zero) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(bias);
  CHECK_BF16(zero);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2, "conv2d_nhwc: x [N,H,W,C], w [Cout,Kp]");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const int64_t Cout = w.size(0), Kp = w.size(1);
  TORCH_CHECK(Cin >= 8 && (Cin & (Cin - 1)) == 0, "conv2d_nhwc: Cin must be a power of two >= 8");
  TORCH_CHECK((kh == kw && (kh == 1 || kh == 3 || kh == 7)) || (kh == 7 && kw == 4),
              "conv2d_nhwc: kernel 1x1, 3x3, 7x7 or 7x4");
  TORCH_CHECK(stride >= 1 && stride_w >= 1 && pad >= 0 && pad_w >= 0, "conv2d_nhwc: stride / pad");
  TORCH_CHECK(Kp % 32 == 0 && Kp >= kh * kw * Cin, "conv2d_nhwc: Kp must cover KH*KW*Cin, multiple of 32");
  TORCH_CHECK(bias.numel() == Cout && zero.numel() >= 8, "conv2d_nhwc: bias / zero page");
  const int64_t bn = tile == 1 ? 64 : 128;
  TORCH_CHECK(tile >= 0 && tile <= 2 && Cout % bn == 0, "conv2d_nhwc: Cout must be a multiple of the tile width");
  const int64_t Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad_w - kw) / stride_w + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "conv2d_nhwc: empty output");
  TORCH_CHECK(N * H * W * Cin < (1LL << 31) && N * Ho * Wo < (1LL << 31), "conv2d_nhwc: size");
  for (const Tensor* t : {&x, &w, &zero})
    TORCH_CHECK(((uintptr_t)t->data_ptr()) % 16 == 0, "conv2d_nhwc: 16-byte alignment");
  auto y = at::empty({N, Ho, Wo, Cout}, x.options());
  const caamd::bf16* rp = nullptr;
  if (residual.has_value()) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->sizes() == y.sizes(), "conv2d_nhwc: residual shape");
    TORCH_CHECK(((uintptr_t)residual->data_ptr()) % 16 == 0, "conv2d_nhwc: residual alignment");
    rp = bp(*residual);
  }
  int lcin = 0;
  while ((1LL << lcin) < Cin) ++lcin;
  if (N * Ho * Wo > 0) {
    const hipError_t e = caamd::conv2d_launch(bp(x), bp(w), bp(bias), rp, bp(y), bp(zero), (int)N, (int)H, (int)W,
                                              lcin, (int)Ho, (int)Wo, (int)kh, (int)kw, (int)stride, (int)stride_w,
                                              (int)pad, (int)pad_w, (int)Cout, (int)Kp, relu, (int)tile,
                                              cur_stream());
    TORCH_CHECK(e == hipSuccess, "conv2d_nhwc: launch failed: ", hipGetErrorString(e));
  }
  return y;
}

// uint8 [N, H, W, 3] -> bf16 [N, H, W, 8] (normalised, channels 3..7 zero)
Tensor normalize_pad8(const Tensor& x, std::vector<double> mean, std::vector<double> std) {
  CHECK_GPU(x);
  CHECK_CONTIG(x);
  CHECK_DT(x, at::kByte);
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3 && mean.size() == 3 && std.size() == 3, "normalize_pad8: NHWC C=3");
  TORCH_CHECK(((uintptr_t)x.data_ptr()) % 16 == 0, "normalize_pad8: 16-byte alignment");
  auto out = at::empty({x.size(0), x.size(1), x.size(2), 8}, x.options().dtype(at::kBFloat16));
  float sc[3], bi[3];
  for (int c = 0; c < 3; ++c) {
    sc[c] = (float)(1.0 / (255.0 * std[c]));
    bi[c] = (float)(-mean[c] / std[c]);
  }
  const int64_t npix = x.size(0) * x.size(1) * x.size(2);
  if (npix) caamd::normalize_pad8_launch(x.data_ptr<uint8_t>(), bp(out), npix, sc, bi, cur_stream());
  LAUNCH_CHECK();
  return out;
}

// uint8 [N, H, W, 3] -> bf16 [N, H + 6, (W + 6) / 2, 8]: the pixel-pair stem input
// (3-pixel zero border, RGB + 0 per pixel, two pixels per 16-byte virtual pixel)
Tensor normalize_pairs(const Tensor& x, std::vector<double> mean, std::vector<double> std) {
  CHECK_GPU(x);
  CHECK_CONTIG(x);
  CHECK_DT(x, at::kByte);
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3 && mean.size() == 3 && std.size() == 3, "normalize_pairs: NHWC C=3");
  TORCH_CHECK(x.size(2) % 2 == 0, "normalize_pairs: even width");
  auto out = at::empty({x.size(0), x.size(1) + 6, (x.size(2) + 6) / 2, 8}, x.options().dtype(at::kBFloat16));
  float sc[3], bi[3];
  for (int c = 0; c < 3; ++c) {
    sc[c] = (float)(1.0 / (255.0 * std[c]));
    bi[c] = (float)(-mean[c] / std[c]);
  }
  if (out.numel())
    caamd::normalize_pairs_launch(x.data_ptr<uint8_t>(), bp(out), (int)x.size(0), (int)x.size(1), (int)x.size(2), sc,
                                  bi, cur_stream());
  LAUNCH_CHECK();
  return out;
}

// 3x3 / stride 2 / pad 1 max pool on bf16 [N, H, W, C] (C % 8 == 0)
Tensor maxpool3s2_nhwc(const Tensor& x) {
  CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "maxpool3s2: [N,H,W,C], C % 8");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  if (y.numel()) caamd::maxpool3s2_launch(bp(x), bp(y), (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, cur_stream());
  LAUNCH_CHECK();
  return y;
}

void add_relu_(Tensor& y, const Tensor& r) {
  CHECK_GPU(y);
  CHECK_GPU(r);
  CHECK_DT(y, at::kBFloat16);
  CHECK_DT(r, at::kBFloat16);
  TORCH_CHECK(y.sizes() == r.sizes() && y.strides() == r.strides(), "add_relu_: shape/stride mismatch");
  TORCH_CHECK(y.is_non_overlapping_and_dense(), "add_relu_: y must be dense");
  TORCH_CHECK(y.numel() % 8 == 0, "add_relu_: numel must be a multiple of 8");
  TORCH_CHECK(((uintptr_t)y.data_ptr()) % 16 == 0 && ((uintptr_t)r.data_ptr()) % 16 == 0,
              "add_relu_: 16-byte alignment");
  if (y.numel()) caamd::add_relu_launch(bp(y), bp(r), y.numel(), cur_stream());
  LAUNCH_CHECK();
}

// ---- hand-written MFMA GEMM (gemm.hip) ------------------------------------------
// layout 0: a[M,K] b[N,K] (y = x W^T) · 1: a[M,K] b[K,N] (dx = dy W) · 2: a[K,M] b[K,N] (dW = dy^T x)
// epi 0: c = acc(+bias) · 1: c += acc(+bias) · 2: ws[s] = partial (split-K; then reduced into c)
//     3: zout = acc+bias, c = gelu(zout) (layout 0) · 4: c = acc*gelu'(z), dbias += colsum(c) (layout 0)
//     5: b = [gate; up] in 64-row blocks, c [M, N/2] = silu(gate) * up (layout 0)
// bpack: b is in the decode GEMM's packed order (algo 9, layout 0, BN % 128 == 0)
static void gemm_bf16(Tensor a, Tensor b, Tensor c, int64_t layout, int64_t epi, int64_t bm,
                      int64_t bn, c10::optional<Tensor> bias, c10::optional<Tensor> z,
                      c10::optional<Tensor> zout, c10::optional<Tensor> dbias, int64_t splitk,
                      c10::optional<Tensor> ws, bool accumulate, int64_t algo,
                      c10::optional<Tensor> tail_ws, c10::optional<Tensor> tail_cnt, int64_t tail_full,
                      int64_t tail_split, bool bpack) {
  CHECK_BF16(a);
  CHECK_BF16(b);
  CHECK_BF16(c);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm: 2-D operands");
  TORCH_CHECK(layout >= 0 && layout <= 2, "gemm: bad layout");
  const int64_t M = layout == 2 ? a.size(1) : a.size(0);
  const int64_t K = layout == 2 ? a.size(0) : a.size(1);
  const int64_t N = layout == 0 ? b.size(0) : b.size(1);
  const int64_t Kb = layout == 0 ? b.size(1) : b.size(0);
  TORCH_CHECK(Kb == K, "gemm: K mismatch");
  TORCH_CHECK(c.size(0) == M && c.size(1) == (epi == 5 ? N / 2 : N), "gemm: output shape mismatch");
  if (bpack)
    TORCH_CHECK(algo % 10 == 9 && layout == 0 && bn % 128 == 0 && N % 128 == 0,
                "gemm: packed B needs algo 9, layout 0 and 128-row-aligned tiles");
  TORCH_CHECK((bm == 256 && (bn == 256 || bn == 320)) || (bm == 128 && bn == 320), "gemm: tile");
  if (algo == 5 || algo == 15) {  // stream-K / lockstep: ragged M allowed (8-aligned), bf16 / accumulate epilogues
    TORCH_CHECK(M % 8 == 0 && N % bn == 0 && K % 64 == 0, "gemm(stream-K): M%8, N%BN, K%64 must be 0");
    TORCH_CHECK(epi == 0 || epi == 1, "gemm(stream-K): bf16 epilogues only");
    TORCH_CHECK(layout == 2 && bm == 256 && bn == 320, "gemm(stream-K): layout 2 with 256 x 320 tiles");
    TORCH_CHECK(!bias.has_value() && splitk == 1, "gemm(stream-K): no bias / explicit split-K");
  } else {
    TORCH_CHECK(M % bm == 0 && N % bn == 0 && K % 64 == 0, "gemm: M%BM, N%BN, K%64 must be 0");
  }
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "gemm: size");
  TORCH_CHECK(splitk >= 1 && splitk <= K / 64, "gemm: splitk");
  using caamd::bf16;
  const bf16* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N, "gemm: bias size");
    bp = (const bf16*)bias->data_ptr();
  }
  const bf16* zp = nullptr;
  bf16* zop = nullptr;
  float* dbp = nullptr;
  void* cp = c.data_ptr();
  int ek = (int)epi;
  if (epi == 3) {
    TORCH_CHECK(layout == 0 && zout.has_value(), "gemm: bias_gelu needs layout 0 and zout");
    CHECK_BF16(*zout);
    TORCH_CHECK(zout->sizes() == c.sizes(), "gemm: zout shape");
    zop = (bf16*)zout->data_ptr();
  } else if (epi == 4) {
    TORCH_CHECK(layout == 0 && z.has_value() && dbias.has_value(), "gemm: dgelu needs layout 0 (B = W^T), z, dbias");
    CHECK_BF16(*z);
    CHECK_F32(*dbias);
    TORCH_CHECK(z->sizes() == c.sizes() && dbias->numel() == N, "gemm: z / dbias shape");
    zp = (const bf16*)z->data_ptr();
    dbp = dbias->data_ptr<float>();
  } else if (epi == 5) {
    TORCH_CHECK(layout == 0 && bn % 128 == 0 && N % 128 == 0 && bp == nullptr && splitk == 1,
                "gemm: SwiGLU needs layout 0, BN % 128 == 0, no bias, no split-K");
  } else if (epi == 2 || splitk > 1) {
    TORCH_CHECK(ws.has_value(), "gemm: split-K needs a workspace");
    CHECK_F32(*ws);
    TORCH_CHECK(ws->numel() >= splitk * M * N, "gemm: workspace too small");
    TORCH_CHECK(bp == nullptr, "gemm: split-K has no bias epilogue");
    cp = ws->data_ptr();
    ek = 2;
  } else {
    TORCH_CHECK(epi == 0 || epi == 1, "gemm: bad epilogue");
    ek = accumulate ? 1 : 0;
  }
  TORCH_CHECK(splitk == 1 || ek == 2, "gemm: split-K only with the f32 partial epilogue");
  const int lda = (int)a.size(1), ldb = (int)b.size(1), ldc = (int)(epi == 5 ? N / 2 : N);
  float* twp = nullptr;
  int* tcp = nullptr;
  if (algo == 5 || algo == 15) {
    const int64_t tiles = ((M + bm - 1) / bm) * (N / bn);
    const int64_t runs = tail_split;
    TORCH_CHECK(runs >= 1 && runs <= 4096, "gemm(stream-K): 1 <= runs <= 4096");
    TORCH_CHECK(tail_ws.has_value() && tail_cnt.has_value(), "gemm(stream-K): needs slabs and tickets");
    CHECK_F32(*tail_ws);
    TORCH_CHECK(tail_cnt->is_cuda() && tail_cnt->scalar_type() == at::kInt && tail_cnt->is_contiguous(),
                "gemm(stream-K): tickets must be int32");
    TORCH_CHECK(tail_ws->numel() >= 2 * runs * bm * bn, "gemm(stream-K): slab workspace too small");
    TORCH_CHECK(tail_cnt->numel() >= tiles, "gemm(stream-K): too few tickets");
    TORCH_CHECK(tiles * (K / 32) >= runs, "gemm(stream-K): fewer K-steps than runs");
    // tail_full > 0: lockstep split-K over tail_full slices, one run per (slice, tile)
    TORCH_CHECK(tail_full <= 0 || (runs == tiles * tail_full && K / 32 >= tail_full),
                "gemm(stream-K lockstep): runs must be tiles x slices, slices <= K-steps");
    TORCH_CHECK(algo != 15 || tail_full > 1, "gemm(algo 15): the external combine needs a lockstep split");
    twp = tail_ws->data_ptr<float>();
    tcp = tail_cnt->data_ptr<int>();
  } else if (tail_split > 1) {
    const int64_t tiles = (M / bm) * (N / bn);
    TORCH_CHECK(ek != 2 && splitk == 1, "gemm: split tail is for the bf16 epilogues");
    TORCH_CHECK((algo % 10 >= 1 && algo % 10 <= 3) || algo % 10 == 9,
                "gemm: split tail needs a ping-pong algo (1-3) or the full-line kernel (9)");
    TORCH_CHECK(tail_full >= 0 && tail_full < tiles && tail_full % 8 == 0 &&
                    ((tiles - tail_full) * tail_split) % 8 == 0, "gemm: bad tail plan");
    TORCH_CHECK(tail_ws.has_value() && tail_cnt.has_value(), "gemm: split tail needs ws and tickets");
    CHECK_F32(*tail_ws);
    TORCH_CHECK(tail_cnt->is_cuda() && tail_cnt->scalar_type() == at::kInt && tail_cnt->is_contiguous(),
                "gemm: tail tickets must be int32");
    TORCH_CHECK(tail_ws->numel() >= (tiles - tail_full) * tail_split * bm * bn, "gemm: tail workspace too small");
    TORCH_CHECK(tail_cnt->numel() >= tiles - tail_full, "gemm: too few tail tickets");
    TORCH_CHECK((K / 32) >= tail_split, "gemm: tail split deeper than K");
    twp = tail_ws->data_ptr<float>();
    tcp = tail_cnt->data_ptr<int>();
  }
  hipError_t e = caamd::gemm_launch((int)layout, ek, (int)bm, (int)bn, (const bf16*)a.data_ptr(),
                                    (const bf16*)b.data_ptr(), cp, bp, zp, zop, dbp, (int)M, (int)N,
                                    (int)K, lda, ldb, ldc, (int)splitk, (int)algo, cur_stream(),
                                    (int)tail_full, (tail_split > 1 || algo == 5 || algo == 15) ? (int)tail_split : 1, twp, tcp,
                                    bpack ? 1 : 0);
  TORCH_CHECK(e == hipSuccess, "gemm launch failed: ", hipGetErrorString(e));
  if (ek == 2) {
    caamd::gemm_splitk_reduce(ws->data_ptr<float>(), (int)splitk, M * N, (bf16*)c.data_ptr(),
                              (int)M, (int)N, ldc, accumulate, cur_stream());
    LAUNCH_CHECK();
  }
}

// NN GEMM on the TN kernel's schedule (gemm.hip algo 27): c[M,N] = a[M,K] b[K,N] (+ bias),
// a K-major (rows of K), b row-major [K, N] (e.g. a weight W[N_out][K_in] as stored, so the
// dgrad dx = dY W needs no transposed copy); 256 x 320 tiles, no split
static void gemm_nn64(Tensor a, Tensor b, Tensor c, c10::optional<Tensor> bias) {
  CHECK_BF16(a);
  CHECK_BF16(b);
  CHECK_BF16(c);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm_nn64: 2-D operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && c.size(0) == M && c.size(1) == N, "gemm_nn64: shape mismatch");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "gemm_nn64: unit inner strides");
  TORCH_CHECK(M % 256 == 0 && N % 320 == 0 && K % 64 == 0 && K > 0, "gemm_nn64: M%256, N%320, K%64 must be 0");
  TORCH_CHECK(256LL * a.stride(0) * 2 < (1LL << 32) && K * b.stride(0) * 2 < (1LL << 32),
              "gemm_nn64: operands must fit a 32-bit buffer descriptor");
  const caamd::bf16* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "gemm_nn64: bias [N]");
    bp = (const caamd::bf16*)bias->data_ptr();
  }
  hipError_t e = caamd::gemm_nn64_launch((const caamd::bf16*)a.data_ptr(), (const caamd::bf16*)b.data_ptr(),
                                         (caamd::bf16*)c.data_ptr(), bp, (int)M, (int)N, (int)K, (int)a.stride(0),
                                         (int)b.stride(0), (int)c.stride(0), cur_stream());
  TORCH_CHECK(e == hipSuccess, "gemm_nn64 launch failed: ", hipGetErrorString(e));
}

// TN weight gradient on the full-line kernel (gemm.hip algo 25): c[M,N] (+)= a[K,M]^T b[K,N],
// 256- or 192-row tiles x 320 columns, lockstep split over `slices` (ws: slices x tiles fp32 slabs)
static void gemm_tn64(Tensor a, Tensor b, Tensor c, int64_t bm, bool accumulate, int64_t slices,
                      c10::optional<Tensor> ws, c10::optional<Tensor> tickets) {
  CHECK_BF16(a);
  CHECK_BF16(b);
  CHECK_BF16(c);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm_tn64: 2-D operands");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && c.size(0) == M && c.size(1) == N, "gemm_tn64: shape mismatch");
  TORCH_CHECK(bm == 256 || bm == 192, "gemm_tn64: bm must be 256 or 192");
  TORCH_CHECK(M % 8 == 0 && M >= 8 && N % 320 == 0 && K % 64 == 0 && K > 0, "gemm_tn64: M%8, N%320, K%64 must be 0");
  TORCH_CHECK(K < (1 << 20) && (int64_t)K * a.size(1) * 2 < (1LL << 32) && (int64_t)K * b.size(1) * 2 < (1LL << 32),
              "gemm_tn64: operands must fit a 32-bit buffer descriptor");
  TORCH_CHECK(slices >= 1 && slices <= K / 64, "gemm_tn64: 1 <= slices <= K/64");
  const int64_t tiles = ((M + bm - 1) / bm) * (N / 320);
  float* wp = nullptr;
  if (slices > 1) {
    TORCH_CHECK(ws.has_value(), "gemm_tn64: split needs a slab workspace");
    CHECK_F32(*ws);
    TORCH_CHECK(ws->numel() >= slices * tiles * bm * 320, "gemm_tn64: slab workspace too small");
    wp = ws->data_ptr<float>();
  }
  int* tp = nullptr;
  if (tickets.has_value() && slices == 2) {  // in-kernel last-arriver combine (two slices); tickets zero between launches
    TORCH_CHECK(tickets->is_cuda() && tickets->scalar_type() == at::kInt && tickets->is_contiguous() &&
                    tickets->numel() >= tiles, "gemm_tn64: tickets must be >= tiles contiguous int32");
    TORCH_CHECK(slices * tiles * bm * 320 * 4 < (1LL << 32), "gemm_tn64: slabs must fit a 32-bit descriptor");
    tp = tickets->data_ptr<int>();
  }
  hipError_t e = caamd::gemm_tn64_launch((int)bm, accumulate, (const caamd::bf16*)a.data_ptr(),
                                         (const caamd::bf16*)b.data_ptr(), (caamd::bf16*)c.data_ptr(), (int)M,
                                         (int)N, (int)K, (int)a.size(1), (int)b.size(1), (int)c.size(1),
                                         (int)slices, wp, cur_stream(), tp);
  TORCH_CHECK(e == hipSuccess, "gemm_tn64 launch failed: ", hipGetErrorString(e));
}

// ---- decode GEMM v3 (decode_gemm.hip): y = x . w^T for M <= 128, weight-streaming --------
// epi 0: y = acc · 1: y = acc + residual · 2: SwiGLU over 64-row-interleaved gate/up weights
// (y has N/2 columns)
// ssp (optional): RMSNorm folded in — per-row sums of squares workspace
// (>= (N/128) * splits * 128 floats); rows of x are scaled by rsqrt(mean(x^2) + eps),
// the norm weight is expected folded into w's columns.
static float* ssp_ptr(const c10::optional<Tensor>& ssp, int64_t need) {
  if (!ssp.has_value()) return nullptr;
  TORCH_CHECK(ssp->is_cuda() && ssp->scalar_type() == at::kFloat && ssp->numel() >= need,
              "decode_gemm: row-statistics workspace too small");
  return ssp->data_ptr<float>();
}

static void decode_gemm(const Tensor& x, const Tensor& w, Tensor& y, c10::optional<Tensor> residual,
                        Tensor& part, Tensor& tick, int64_t epi, int64_t splits, bool packed,
                        c10::optional<Tensor> ssp, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(y);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "decode_gemm: 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && w.is_contiguous(), "decode_gemm: w must be a contiguous [N, K]");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) >= K, "decode_gemm: x rows must be dense");
  TORCH_CHECK(M >= 1 && M <= 128, "decode_gemm: 1 <= M <= 128");
  TORCH_CHECK(N % 128 == 0 && K % 64 == 0, "decode_gemm: N % 128 == 0, K % 64 == 0");
  TORCH_CHECK(epi >= 0 && epi <= 2, "decode_gemm: epi 0, 1 or 2");
  const int64_t NY = epi == 2 ? N / 2 : N;
  TORCH_CHECK(y.size(0) == M && y.size(1) == NY && y.stride(1) == 1, "decode_gemm: y shape");
  TORCH_CHECK(splits >= 1 && K % 64 == 0 && (splits - 1) * ((K / 64 + splits - 1) / splits) < K / 64,
              "decode_gemm: K % 64 == 0 and every split non-empty");
  const caamd::bf16* rp = nullptr;
  if (epi == 1) {
    TORCH_CHECK(residual.has_value(), "decode_gemm: residual epilogue needs a residual");
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->sizes() == y.sizes() && residual->stride(0) == y.stride(0) && residual->stride(1) == 1,
                "decode_gemm: residual must match y");
    rp = (const caamd::bf16*)residual->data_ptr();
  }
  if (splits > 1) {
    TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.numel() >= (N / 128) * splits * 16384,
                "decode_gemm: partial workspace too small");
    TORCH_CHECK(tick.is_cuda() && tick.scalar_type() == at::kInt && tick.numel() >= N / 128,
                "decode_gemm: tickets too small");
  }
  hipError_t e = caamd::decode_gemm_launch((int)epi, (const caamd::bf16*)x.data_ptr(), (const caamd::bf16*)w.data_ptr(),
                                           (caamd::bf16*)y.data_ptr(), rp, part.data_ptr<float>(),
                                           reinterpret_cast<unsigned*>(tick.data_ptr<int>()), (int)M, (int)N, (int)K,
                                           (int)x.stride(0), (int)y.stride(0), (int)splits, packed,
                                           ssp_ptr(ssp, (N / 128) * splits * 128), (float)eps, cur_stream());
  TORCH_CHECK(e == hipSuccess, "decode_gemm launch failed: ", hipGetErrorString(e));
}

// o / down projection on the decode GEMM (w prepacked, splits > 1) with the split-K
// combine, the residual add (res updated in place) and the next RMSNorm in one launch:
// returns h = rmsnorm(res + x . w^T) * norm_w.
static Tensor decode_gemm_norm(const Tensor& x, const Tensor& w, Tensor& part, int64_t splits, Tensor& res,
                               const Tensor& norm_w, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(res);
  CHECK_BF16(norm_w);
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) >= K && w.size(1) == K && w.is_contiguous(),
              "decode_gemm_norm: x, w");
  TORCH_CHECK(M >= 1 && M <= 128 && K % 64 == 0 && N % 128 == 0 && N <= 8192, "decode_gemm_norm: shapes");
  TORCH_CHECK(res.dim() == 2 && res.size(0) == M && res.size(1) == N && res.is_contiguous(), "decode_gemm_norm: res");
  TORCH_CHECK(norm_w.numel() == N && norm_w.is_contiguous(), "decode_gemm_norm: norm weight");
  TORCH_CHECK(splits >= 2 && (splits - 1) * ((K / 64 + splits - 1) / splits) < K / 64,
              "decode_gemm_norm: 2 <= splits, every split non-empty");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.numel() >= splits * 128 * N,
              "decode_gemm_norm: partial workspace too small");
  Tensor h = torch::empty({M, N}, res.options());
  hipError_t e = caamd::decode_gemm_norm_launch(
      (const caamd::bf16*)x.data_ptr(), (const caamd::bf16*)w.data_ptr(), part.data_ptr<float>(), (int)M, (int)N,
      (int)K, (int)x.stride(0), (int)splits, (caamd::bf16*)res.data_ptr(), (const caamd::bf16*)norm_w.data_ptr(),
      (caamd::bf16*)h.data_ptr(), (float)eps, cur_stream());
  TORCH_CHECK(e == hipSuccess, "decode_gemm_norm launch failed: ", hipGetErrorString(e));
  return h;
}

// qkv projection on the decode GEMM (w prepacked, head_dim 128, splits > 1) with
// RoPE and the paged-cache append fused into the split-K reduce launch:
// y = rope(x . w^T); k / v rows of y also written to their cache slots.
static void decode_gemm_qkv_rope(const Tensor& x, const Tensor& w, Tensor& y, Tensor& part, int64_t splits,
                                 const Tensor& cos_sin, const Tensor& positions, const Tensor& slots,
                                 const Tensor& k_cache, const Tensor& v_cache, int64_t H, int64_t KVH,
                                 c10::optional<Tensor> ssp, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(y);
  CHECK_F32(cos_sin);
  CHECK_BF16(k_cache);
  CHECK_BF16(v_cache);
  for (const Tensor* t : {&positions, &slots}) {
    CHECK_GPU(*t);
    CHECK_CONTIG(*t);
    CHECK_DT(*t, at::kInt);
  }
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.size(1) == K && w.is_contiguous(), "decode_gemm_qkv_rope: x, w");
  TORCH_CHECK(M >= 1 && M <= 128 && K % 64 == 0 && N == (H + 2 * KVH) * 128, "decode_gemm_qkv_rope: shapes");
  TORCH_CHECK(y.dim() == 2 && y.size(0) == M && y.size(1) == N && y.stride(1) == 1, "decode_gemm_qkv_rope: y");
  TORCH_CHECK(splits >= 2 && K % 64 == 0 && (splits - 1) * ((K / 64 + splits - 1) / splits) < K / 64,
              "decode_gemm_qkv_rope: 2 <= splits, K % 64 == 0, every split non-empty");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.numel() >= (N / 128) * splits * 16384,
              "decode_gemm_qkv_rope: partial workspace too small");
  TORCH_CHECK(cos_sin.dim() == 3 && cos_sin.size(1) == 64 && cos_sin.size(2) == 2, "decode_gemm_qkv_rope: cos_sin");
  TORCH_CHECK(positions.numel() == M && slots.numel() == M, "decode_gemm_qkv_rope: positions / slots");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == KVH && k_cache.size(3) == 128 &&
                  v_cache.sizes() == k_cache.sizes() && k_cache.is_contiguous() && v_cache.is_contiguous(),
              "decode_gemm_qkv_rope: cache must be [num_blocks, KVH, BS, 128]");
  hipError_t e = caamd::decode_gemm_qkv_rope_launch(
      (const caamd::bf16*)x.data_ptr(), (const caamd::bf16*)w.data_ptr(), (caamd::bf16*)y.data_ptr(),
      part.data_ptr<float>(), (int)M, (int)N, (int)K, (int)x.stride(0), (int)y.stride(0), (int)splits,
      cos_sin.data_ptr<float>(), positions.data_ptr<int>(), slots.data_ptr<int>(), bp(k_cache), bp(v_cache), (int)H,
      (int)KVH, (int)k_cache.size(2), ssp_ptr(ssp, (N / 128) * splits * 128), (float)eps, cur_stream());
  TORCH_CHECK(e == hipSuccess, "decode_gemm_qkv_rope launch failed: ", hipGetErrorString(e));
}

static Tensor transpose_bf16(const Tensor& x) {
  CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && x.size(0) % 64 == 0 && x.size(1) % 64 == 0, "transpose: [R,C] with R,C % 64 == 0");
  auto y = at::empty({x.size(1), x.size(0)}, x.options());
  if (x.numel() > 0) {
    caamd::transpose_bf16((const caamd::bf16*)x.data_ptr(), (caamd::bf16*)y.data_ptr(), (int)x.size(0),
                          (int)x.size(1), cur_stream());
    LAUNCH_CHECK();
  }
  return y;
}

// ---- RLlib encoder / PPO loss (rl_encoder.hip) ------------------------------------
static inline bool aligned16(const Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

// layout 0: C[M,N] = A[M,K] . B[N,K]^T ; 1: A[M,K] . B[K,N] ; 2: A[K,M]^T . B[K,N]
void rl_gemm_(const Tensor& a, const Tensor& b, const Tensor& c, int64_t layout, int64_t epi,
              std::optional<Tensor> bias, std::optional<Tensor> aux, int64_t M, int64_t N, int64_t K,
              int64_t lda, int64_t ldb, int64_t ldc, int64_t splits) {
  CHECK_BF16(a);
  CHECK_BF16(b);
  CHECK_GPU(c);
  CHECK_CONTIG(c);
  TORCH_CHECK(layout >= 0 && layout <= 2, "rl_gemm: layout must be 0, 1 or 2");
  TORCH_CHECK(epi >= 0 && epi <= 5, "rl_gemm: bad epilogue");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31),
              "rl_gemm: bad sizes");
  TORCH_CHECK(aligned16(a) && aligned16(b), "rl_gemm: operands must be 16-byte aligned");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "rl_gemm: leading dims must be multiples of 8 (c: 4)");
  // the contiguous dim of every operand is read in 8-element vectors
  const int64_t a_vec = layout == 2 ? M : K, b_vec = layout == 0 ? K : N;
  TORCH_CHECK(a_vec % 8 == 0 && b_vec % 8 == 0 && N % 4 == 0, "rl_gemm: vector dims must be multiples of 8");
  const int64_t a_need = layout == 2 ? (K - 1) * lda + M : (M - 1) * lda + K;
  const int64_t b_need = layout == 0 ? (N - 1) * ldb + K : (K - 1) * ldb + N;
  TORCH_CHECK(a.numel() >= a_need && b.numel() >= b_need, "rl_gemm: operand too small for M/N/K/ld");
  TORCH_CHECK(c.numel() >= (M - 1) * ldc + N, "rl_gemm: output too small");
  TORCH_CHECK(c.scalar_type() == (epi == 3 ? at::kFloat : at::kBFloat16),
              "rl_gemm: c must be fp32 for the atomic epilogue, bf16 otherwise");
  const caamd::bf16* bp = nullptr;
  const caamd::bf16* xp = nullptr;
  if (bias && bias->defined()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() >= N, "rl_gemm: bias too small");
    bp = reinterpret_cast<const caamd::bf16*>(bias->data_ptr());
  }
  if (epi == 4 || epi == 5) {
    TORCH_CHECK(aux && aux->defined(), "rl_gemm: activation-backward epilogue needs aux");
    CHECK_BF16(*aux);
    TORCH_CHECK(aux->numel() >= (M - 1) * ldc + N, "rl_gemm: aux too small");
    xp = reinterpret_cast<const caamd::bf16*>(aux->data_ptr());
  }
  caamd::rl_gemm((int)layout, reinterpret_cast<const caamd::bf16*>(a.data_ptr()),
                 reinterpret_cast<const caamd::bf16*>(b.data_ptr()), c.data_ptr(), bp, xp, (int)M, (int)N, (int)K,
                 (int)lda, (int)ldb, (int)ldc, (int)epi, (int)std::max<int64_t>(1, splits), cur_stream());
  LAUNCH_CHECK();
}

static void check_conv_geom(int64_t B, int64_t H, int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t S) {
  TORCH_CHECK(B > 0 && H >= KH && W >= KW && KH > 0 && KW > 0 && S > 0 && C > 0, "rl conv: bad geometry");
  TORCH_CHECK((KW * C) % 8 == 0 && (S * C) % 8 == 0 && (W * C) % 8 == 0,
              "rl conv: KW*C, S*C and W*C must be multiples of 8");
}

void rl_im2col_(const Tensor& x, const Tensor& col, int64_t KH, int64_t KW, int64_t S, double scale) {
  CHECK_GPU(x);
  CHECK_CONTIG(x);
  CHECK_BF16(col);
  TORCH_CHECK(x.dim() == 4, "rl_im2col: x must be NHWC");
  const bool u8 = x.scalar_type() == at::kByte;
  TORCH_CHECK(u8 || x.scalar_type() == at::kBFloat16, "rl_im2col: x must be uint8 or bf16");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  check_conv_geom(B, H, W, C, KH, KW, S);
  const int64_t OH = (H - KH) / S + 1, OW = (W - KW) / S + 1;
  TORCH_CHECK(col.numel() == B * OH * OW * KH * KW * C, "rl_im2col: col must be [B*OH*OW, KH*KW*C]");
  TORCH_CHECK(aligned16(col) && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, "rl_im2col: alignment");
  caamd::rl_im2col(x.data_ptr(), u8, reinterpret_cast<caamd::bf16*>(col.data_ptr()), (int)B, (int)H, (int)W,
                   (int)C, (int)KH, (int)KW, (int)S, (float)scale, cur_stream());
  LAUNCH_CHECK();
}

void rl_col2im_(const Tensor& dcol, std::optional<Tensor> y, const Tensor& dz, int64_t KH, int64_t KW, int64_t S,
                int64_t act) {
  CHECK_BF16(dcol);
  CHECK_BF16(dz);
  TORCH_CHECK(dz.dim() == 4, "rl_col2im: dz must be NHWC");
  const int64_t B = dz.size(0), H = dz.size(1), W = dz.size(2), C = dz.size(3);
  check_conv_geom(B, H, W, C, KH, KW, S);
  TORCH_CHECK(C % 8 == 0, "rl_col2im: C must be a multiple of 8");
  const int64_t OH = (H - KH) / S + 1, OW = (W - KW) / S + 1;
  TORCH_CHECK(dcol.numel() == B * OH * OW * KH * KW * C, "rl_col2im: dcol must be [B*OH*OW, KH*KW*C]");
  TORCH_CHECK(act >= 0 && act <= 2, "rl_col2im: act must be 0 (none), 1 (relu) or 2 (tanh)");
  const caamd::bf16* yp = nullptr;
  if (act) {
    TORCH_CHECK(y && y->defined(), "rl_col2im: activation mask needs y");
    CHECK_BF16(*y);
    TORCH_CHECK(y->numel() == dz.numel(), "rl_col2im: y must match dz");
    yp = reinterpret_cast<const caamd::bf16*>(y->data_ptr());
  }
  caamd::rl_col2im(reinterpret_cast<const caamd::bf16*>(dcol.data_ptr()), yp,
                   reinterpret_cast<caamd::bf16*>(dz.data_ptr()), (int)B, (int)H, (int)W, (int)C, (int)KH, (int)KW,
                   (int)S, (int)act, cur_stream());
  LAUNCH_CHECK();
}

void rl_colsum_(const Tensor& x, const Tensor& db) {
  CHECK_BF16(x);
  CHECK_F32(db);
  TORCH_CHECK(x.dim() == 2 && db.numel() == x.size(1), "rl_colsum: x [M,N], db [N]");
  TORCH_CHECK(x.size(1) % 8 == 0 && x.size(1) <= 2048 && aligned16(x), "rl_colsum: N must be a multiple of 8, <= 2048");
  if (x.size(0) > 0)
    caamd::rl_colsum(reinterpret_cast<const caamd::bf16*>(x.data_ptr()), db.data_ptr<float>(), (int)x.size(0),
                     (int)x.size(1), cur_stream());
  LAUNCH_CHECK();
}

// returns (dlogits [B,A], dvf [B], stats [4] = sums of surrogate, vf loss, entropy, kl)
std::vector<Tensor> ppo_loss_cat_(const Tensor& logits, const Tensor& vf, const Tensor& actions,
                                  const Tensor& old_logp, const Tensor& adv, const Tensor& vt,
                                  const Tensor& old_logits, double clip, double vf_clip, double vf_coeff,
                                  double ent_coeff, double kl_coeff, std::optional<Tensor> kl_dev) {
  CHECK_F32(logits);
  CHECK_F32(vf);
  CHECK_F32(old_logp);
  CHECK_F32(adv);
  CHECK_F32(vt);
  CHECK_F32(old_logits);
  CHECK_GPU(actions);
  CHECK_CONTIG(actions);
  CHECK_DT(actions, at::kLong);
  TORCH_CHECK(logits.dim() == 2 && old_logits.sizes() == logits.sizes(), "ppo_loss: logits [B,A]");
  const int64_t B = logits.size(0), A = logits.size(1);
  TORCH_CHECK(A > 0 && vf.numel() == B && actions.numel() == B && old_logp.numel() == B && adv.numel() == B &&
                  vt.numel() == B,
              "ppo_loss: per-sample inputs must have B elements");
  const float* klp = nullptr;
  if (kl_dev && kl_dev->defined()) {
    CHECK_F32(*kl_dev);
    TORCH_CHECK(kl_dev->numel() >= 1, "ppo_loss: kl_dev must hold the KL coefficient");
    klp = kl_dev->data_ptr<float>();
  }
  auto dlogits = at::empty_like(logits);
  auto dvf = at::empty_like(vf);
  auto stats = at::zeros({4}, logits.options());
  if (B > 0) {
    // the kernel clamps action indices into [0, A) (no out-of-row reads)
    caamd::ppo_loss_cat(logits.data_ptr<float>(), vf.data_ptr<float>(), actions.data_ptr<int64_t>(),
                        old_logp.data_ptr<float>(), adv.data_ptr<float>(), vt.data_ptr<float>(),
                        old_logits.data_ptr<float>(), (int)B, (int)A, (float)clip, (float)vf_clip, (float)vf_coeff,
                        (float)ent_coeff, (float)kl_coeff, klp, dlogits.data_ptr<float>(), dvf.data_ptr<float>(),
                        stats.data_ptr<float>(), cur_stream());
  }
  LAUNCH_CHECK();
  return {dlogits, dvf, stats};
}

// ---- device guard for every tensor entry point -----------------------------------
// Workers may see several GPUs (Train worker groups run with every GPU of the node
// visible for RCCL P2P), and a tensor need not live on the current device: every
// binding below runs under a HIP device guard set to the device of its GPU tensor
// arguments, after checking that all of them live on ONE device (a launch on the
// current device's stream with another device's pointers would fault or silently
// compute on the wrong GPU). Registered through GUARDED(fn) in PYBIND11_MODULE.
struct DeviceSel {
  int index = -1;
  void see_device(bool is_gpu, int idx, const char* what) {
    if (!is_gpu) return;
    if (index < 0) {
      index = idx;
    } else {
      TORCH_CHECK(idx == index, "kernel arguments live on different GPUs (", what, " is on cuda:", idx,
                  ", an earlier tensor on cuda:", index, ")");
    }
  }
  void see(const Tensor& t) {
    if (t.defined()) see_device(t.is_cuda(), t.is_cuda() ? (int)t.get_device() : -1, "a tensor");
  }
  void see(const c10::optional<Tensor>& t) {
    if (t.has_value()) see(*t);
  }
  void see(const std::vector<Tensor>& ts) {
    for (const auto& t : ts) see(t);
  }
  template <typename T>
  void see(const T&) {}
};

template <auto F>
struct GuardedCall;
template <typename R, typename... A, R (*F)(A...)>
struct GuardedCall<F> {
  static R call(A... a) {
    DeviceSel sel;
    (sel.see(a), ...);
    c10::hip::OptionalHIPGuard guard;
    if (sel.index >= 0) guard.set_index((c10::DeviceIndex)sel.index);
    return F(std::forward<A>(a)...);
  }
};
#define GUARDED(f) (&GuardedCall<&f>::call)

// CPU-testable form of the selection rule: [(is_gpu, index)] -> chosen index (-1: none)
static int64_t select_device_(const std::vector<std::pair<bool, int64_t>>& devs) {
  DeviceSel sel;
  for (const auto& d : devs) sel.see_device(d.first, (int)d.second, "an argument");
  return sel.index;
}

PYBIND11_MODULE(_C, m) {
  m.def("_select_device", &select_device_);
  m.doc() = "cluster_anywhere_amd gfx950 HIP kernels";
  m.def("gemm_bf16", GUARDED(gemm_bf16), pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("c"),
        pybind11::arg("layout"), pybind11::arg("epi"), pybind11::arg("bm"), pybind11::arg("bn"),
        pybind11::arg("bias"), pybind11::arg("z"), pybind11::arg("zout"), pybind11::arg("dbias"),
        pybind11::arg("splitk"), pybind11::arg("ws"), pybind11::arg("accumulate"),
        pybind11::arg("algo") = 1, pybind11::arg("tail_ws") = pybind11::none(),
        pybind11::arg("tail_cnt") = pybind11::none(), pybind11::arg("tail_full") = -1,
        pybind11::arg("tail_split") = 1, pybind11::arg("bpack") = false);
  m.def("gemm_tn64", GUARDED(gemm_tn64), pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("c"),
        pybind11::arg("bm"), pybind11::arg("accumulate"), pybind11::arg("slices"),
        pybind11::arg("ws") = pybind11::none(), pybind11::arg("tickets") = pybind11::none());
  m.def("gemm_nn64", GUARDED(gemm_nn64), pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("c"),
        pybind11::arg("bias") = pybind11::none());
  m.def("gemm_set_tail_first", [](int64_t v) { caamd::gemm_set_tail_first((int)v); });
  m.def("gemm_set_tn_group_m", [](int64_t g) {  // m-tiles per tile-order group of the TN wgrad kernel (0: 8)
    TORCH_CHECK(g >= 0 && g <= 64, "gemm_set_tn_group_m: 0..64");
    caamd::gemm_set_tn_group_m((int)g);
  });
  m.def("gemm_set_group_m", [](int64_t g) {  // m-tiles per tile-order group of the k64 kernel (0: 8)
    TORCH_CHECK(g >= 0 && g <= 64, "gemm_set_group_m: 0..64");
    caamd::gemm_set_group_m((int)g);
  });
  m.def("gemm_tail_plan", [](int64_t tiles, int64_t K, int64_t ks, int64_t slots, int64_t max_split) {
    int full, S;
    caamd::gemm_tail_plan((int)tiles, (int)K, (int)ks, (int)slots, (int)max_split, &full, &S);
    return std::vector<int64_t>{full, S};
  });
  m.def("decode_gemm", GUARDED(decode_gemm));
  m.def("decode_gemm_qkv_rope", GUARDED(decode_gemm_qkv_rope));
  m.def("decode_gemm_norm", GUARDED(decode_gemm_norm));
  m.def("decode_gemm_config", [](int64_t ext) { caamd::decode_gemm_config((int)ext); });
  m.def("transpose_bf16", GUARDED(transpose_bf16));
  m.def("layernorm_fwd", GUARDED(layernorm_fwd));
  m.def("layernorm_bwd", GUARDED(layernorm_bwd), pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("g"),
        pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("dres"), pybind11::arg("dxsum") = pybind11::none(),
        pybind11::arg("g_main") = pybind11::none(), pybind11::arg("b_main") = pybind11::none());
  m.def("ln_bwd_dxsum_ok", [](int64_t D) { return caamd::ln_bwd_dxsum_ok((int)D); });
  m.def("ln_bwd_config", [](int variant, int max_blocks) {
    TORCH_CHECK(variant >= 0 && variant <= 3, "ln_bwd_config: variant must be 0-3");
    TORCH_CHECK(max_blocks >= 0 && max_blocks <= 65536, "ln_bwd_config: bad max_blocks");
    caamd::ln_bwd_config(variant, max_blocks);
  });
  m.def("bias_gelu_fwd", GUARDED(bias_gelu_fwd));
  m.def("bias_gelu_bwd", GUARDED(bias_gelu_bwd));
  m.def("bias_grad_", GUARDED(bias_grad_));
  m.def("drain_f32_", GUARDED(drain_f32_));
  m.def("xent_fwd", GUARDED(xent_fwd));
  m.def("xent_bwd_", GUARDED(xent_bwd_));
  m.def("xent_fused_", GUARDED(xent_fused_));
  m.def("grad_sumsq", GUARDED(grad_sumsq));
  m.def("adamw_config", [](int64_t variant) { caamd::adamw_config((int)variant); });
  m.def("fa64_set_pair", [](int64_t v) { caamd::fa64_set_pair((int)v); });
  m.def("adamw_step", GUARDED(adamw_step));
  m.def("gae", GUARDED(gae));
  m.def("vtrace", GUARDED(vtrace));
  m.def("flash_attn_fwd", GUARDED(flash_attn_fwd));
  m.def("flash_attn_bwd", GUARDED(flash_attn_bwd), pybind11::arg("qkv"), pybind11::arg("out"), pybind11::arg("dout"),
        pybind11::arg("lse"), pybind11::arg("H"), pybind11::arg("causal"), pybind11::arg("dbias") = pybind11::none());
  m.def("rmsnorm", GUARDED(rmsnorm), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("eps"),
        pybind11::arg("residual") = pybind11::none());
  m.def("silu_mul", GUARDED(silu_mul));
  m.def("argmax_rows", GUARDED(argmax_rows));
  m.def("rope_cache_", GUARDED(rope_cache_));
  m.def("paged_decode", GUARDED(paged_decode), pybind11::arg("q"), pybind11::arg("k_cache"), pybind11::arg("v_cache"),
        pybind11::arg("block_tables"), pybind11::arg("ctx_lens"), pybind11::arg("max_ctx"), pybind11::arg("H"),
        pybind11::arg("scale"), pybind11::arg("impl") = -1);
  m.def("flash_attn_gqa", GUARDED(flash_attn_gqa));
  m.def("image_normalize", GUARDED(image_normalize));
  m.def("add_relu_", GUARDED(add_relu_));
  m.def("conv2d_nhwc", GUARDED(conv2d_nhwc));
  m.def("conv2d_nhwc_ex", GUARDED(conv2d_nhwc_ex));
  m.def("normalize_pad8", GUARDED(normalize_pad8));
  m.def("normalize_pairs", GUARDED(normalize_pairs));
  m.def("maxpool3s2_nhwc", GUARDED(maxpool3s2_nhwc));
  m.def("bias_act_", GUARDED(bias_act_));
  m.def("rl_gemm", GUARDED(rl_gemm_));
  m.def("rl_im2col", GUARDED(rl_im2col_));
  m.def("rl_col2im", GUARDED(rl_col2im_));
  m.def("rl_colsum", GUARDED(rl_colsum_));
  m.def("ppo_loss_cat", GUARDED(ppo_loss_cat_));
}
