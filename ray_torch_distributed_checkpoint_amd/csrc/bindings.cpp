// Python bindings for the MI355X kernels and the native checkpoint engine.
//
// Kernels live in lean .hip translation units exposing extern "C" launchers (raw pointers +
// hipStream_t); this file is the only one that includes the torch headers.  Every launcher
// runs on the caller's current HIP stream so ops compose with torch stream semantics and
// hipGraph capture.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <pybind11/stl.h>

#include "kernels/args.h"
#include "runtime/ckpt_engine.cpp"
#include "runtime/reducer.cpp"

using torch::Tensor;
namespace py = pybind11;

extern "C" {
int rtdc_gemm_bf16(const rtdc::GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int batch,
                   hipStream_t stream, int* cs_rows_out);
int rtdc_gemm_f32(const rtdc::GemmF32Args* args, hipStream_t st);
int rtdc_gemm8_grouped(const rtdc::GemmArgs* args, int n, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st);
int rtdc_gemm4b_set(int v);
int rtdc_conv_gemm(const rtdc::GemmArgs* args, int mode, hipStream_t stream);
int rtdc_layernorm_fwd(const void* x, const void* g, const void* b, void* y, float* mean, float* rstd,
                       int M, int D, float eps, hipStream_t st);
int rtdc_rmsnorm_fwd(const void* x, const void* g, void* y, float* rstd, int M, int D, float eps,
                     hipStream_t st);
int rtdc_layernorm_bwd(const void* dy, const void* x, const void* g, const float* mean, const float* rstd,
                       const void* dres, void* dx, float* ws, float* dg, float* db, float* dxsum, int M, int D,
                       int nwaves, int accumulate, hipStream_t st, int* nblk_out);
int rtdc_rmsnorm_bwd(const void* dy, const void* x, const void* g, const float* rstd, const void* dres,
                     void* dx, float* ws, float* dg, float* dxsum, int M, int D, int nwaves, int accumulate,
                     hipStream_t st);
int rtdc_colsum(const void* X, int M, int N, int ld, float* ws, int nblk, float* out, int accumulate,
                int is_bf16, hipStream_t st);
int rtdc_colsum_partial(const void* X, int M, int N, int ld, float* ws, int nblk, int is_bf16, hipStream_t st);
int rtdc_colsum_multi(const float* const* ws, float* const* out, const int* W, const int* D, const int* accumulate,
                      int n, hipStream_t st);
int rtdc_xent(const void* logits, void* dlogits, const int64_t* target, float* loss, float* lse,
              int64_t* argmax, int M, int V, int ld, float grad_scale, int ignore_index, int is_bf16,
              hipStream_t st);
int rtdc_adamw(const void* chunks, int nchunks, float* p, const float* g, float* m, float* v, void* shadow,
               float lr, float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt,
               float grad_scale, const int* skip, hipStream_t st);
int rtdc_sgd(const void* chunks, int nchunks, float* p, const float* g, float* buf, void* shadow, float lr,
             float momentum, float dampening, float wd, int nesterov, int first, float grad_scale,
             const int* skip, hipStream_t st);
int rtdc_f32_to_bf16(const float* x, void* y, long long n, hipStream_t st);
int rtdc_f32_to_bf16_t(const float* x, void* y, int R, int C, hipStream_t st);
int rtdc_bf16_transpose_multi(const void* const* src, void* const* dst, const int* R, const int* C, int n,
                              void* jobs_dev, hipStream_t st);
int rtdc_bf16_transpose_jobs_bytes();
int rtdc_sumsq(const void* chunks, int nchunks, const float* g, float* partial, hipStream_t st);
int rtdc_softmax_fwd(const void* S, void* P, float* lse, long long rows, int T, int causal, hipStream_t st);
int rtdc_softmax_bwd(const void* P, const void* dP, void* dS, long long rows, int T, int causal,
                     hipStream_t st);
int rtdc_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int ntok, int T, int D,
                   hipStream_t st);
int rtdc_sort_ids(const int64_t* ids, int n, int nbits, uint32_t* ws, int64_t* sorted, int64_t* perm,
                  hipStream_t st);
int rtdc_synth_tokens(const int64_t* ids, int B, int T, long long vocab, unsigned long long seed_add, int64_t* inp,
                      int64_t* tgt, hipStream_t st);
int rtdc_fill_f32(float* x, long long n, float v, hipStream_t st);
int rtdc_embed_bwd(const int64_t* sidx, const int64_t* perm, const void* dout, float* dwte, float* dwpe, int B, int T,
                   int D, int accumulate_wpe, int accumulate_wte, hipStream_t st);
int rtdc_dropout(const void* x, void* y, long long n, float p, unsigned long long seed,
                 unsigned long long offset, const long long* off_dev, int is_bf16, hipStream_t st);
int rtdc_relu_dropout(const void* h, void* y, const void* dy, void* dx, long long n, float p,
                      unsigned long long seed, unsigned long long offset, int backward, int is_bf16,
                      hipStream_t st);
int rtdc_flash_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, int Hkv, int Dh, float scale,
                   hipStream_t st);
int rtdc_rope(const void* x, void* y, const float* cosb, const float* sinb, int ntok, int T, int nrot_heads,
              int ntot_heads, int Dh, int inverse, hipStream_t st);
int rtdc_swiglu_fwd(const void* gu, void* h, long long M, int F, hipStream_t st);
int rtdc_swiglu_bwd(const void* gu, const void* dh, void* dgu, long long M, int F, hipStream_t st);
int rtdc_im2col(const void* x, void* cols, int B, int H, int W, int C, int Ho, int Wo, int KH, int KW, int stride,
                int pad, int K, int Kp, hipStream_t st);
int rtdc_xent_finalize(const float* loss, const int64_t* target, int M, float fixed_n, int ignore, float* out,
                       hipStream_t st);
int rtdc_xent_alpha(const float* g, const float* den, float* out, hipStream_t st);
int rtdc_scale_dev(const void* x, void* y, long long n, int is_bf16, const float* g, const float* den, hipStream_t st);
int rtdc_nchw_to_nhwc_bf16(const float* x, void* y, int B, int C, long long HW, hipStream_t st);
int rtdc_col2im(const void* dcols, void* dx, const void* addend, int B, int H, int W, int C, int Ho, int Wo, int KH,
                int KW, int stride, int pad, int K, int Kp, hipStream_t st);
int rtdc_bn_fwd(const void* x, const void* res, void* y, float* mean, float* rstd, const float* gamma, const float* beta,
                float* running_mean, float* running_var, long long N, int C, float eps, float momentum, int training,
                int relu, float* ws, int nblk, const float* pmean, const float* pm2, int p_nblk, int p_R,
                long long* nbt, hipStream_t st);
int rtdc_conv_w_flip_t(const void* w, void* out, int Cout, int KH, int KW, int C, hipStream_t st);
int rtdc_stem_s2d(const float* x, void* y, int B, int H, int W, hipStream_t st);
int rtdc_stem_w_s2d(const void* w, void* wp, int Cout, hipStream_t st);
int rtdc_stem_dw_s2d(const float* dwp, float* dw, int Cout, hipStream_t st);
int rtdc_bn_relu_maxpool(const void* x, void* y, void* arg, const float* mean, const float* rstd, const float* gamma,
                         const float* beta, int B, int H, int W, int C, int Ho, int Wo, int K, int s, int p,
                         hipStream_t st);
int rtdc_pool_bn_bwd(const void* dy, const void* arg, const void* x, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, void* dx, float* dgamma, float* dbeta, float* ws, int nblk,
                     int B, int H, int W, int C, int Ho, int Wo, hipStream_t st);
int rtdc_bn_bwd(const void* dy, const void* y, const void* x, const float* mean, const float* rstd, const float* gamma,
                const float* beta, void* dx, void* dres, float* dgamma, float* dbeta, long long N, int C, int relu,
                float* ws, int nblk, const float* psum, const float* psumx, int p_nblk, hipStream_t st);
int rtdc_maxpool(const void* x, void* y, void* arg, const void* dy, void* dx, int B, int H, int W, int C, int Ho, int Wo,
                 int K, int s, int p, int backward, hipStream_t st);
int rtdc_avgpool(const void* x, void* y, int B, int HW, int C, int backward, hipStream_t st);
int rtdc_flash_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv,
                   int B, int T, int H, int Hkv, int Dh, float scale, float* cs_ws, float* part, int qs, int which,
                   int delta_ready, hipStream_t st);
int rtdc_flash_delta(const void* out, const void* dout, float* delta, int B, int T, int H, int Dh, hipStream_t st);
}

static hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

static void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed (rc=", rc, rc == 1 ? ": unsupported shape" : ": launch error", ")");
}

static void* ptr_or_null(const c10::optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

static void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
}

// ---------------------------------------------------------------------------------- GEMMs
// Returns the number of deferred column-sum partial rows left in cs_ws (cs_ws given without
// cs_out: see rtdc_gemm_bf16), else 0.
static int64_t gemm_bf16(Tensor A, Tensor B, Tensor C, c10::optional<Tensor> Cin, c10::optional<Tensor> bias,
                      c10::optional<Tensor> aux_in, c10::optional<Tensor> aux_out, int64_t M, int64_t N,
                      int64_t K, int64_t lda, int64_t ldb, int64_t ldc, bool a_kmajor, bool b_kmajor,
                      int64_t batch, int64_t batch_inner, int64_t sA0, int64_t sA1, int64_t sB0, int64_t sB1,
                      int64_t sC0, int64_t sC1, double alpha, double beta, int64_t act, int64_t causal,
                      c10::optional<Tensor> ws, int64_t tile_cfg, c10::optional<Tensor> alpha_dev,
                      c10::optional<Tensor> cs_out, c10::optional<Tensor> cs_ws) {
  check_dev(A, "A");
  check_dev(B, "B");
  check_dev(C, "C");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "A/B must be bf16");
  TORCH_CHECK(C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat, "C must be bf16/fp32");
  TORCH_CHECK(K % 64 == 0 && M % 8 == 0 && N % 8 == 0, "gemm_bf16: need K%64==0, M%8==0, N%8==0");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "gemm_bf16: leading dims must be 16-B multiples");
  rtdc::GemmArgs a{};
  a.A = (const uint16_t*)A.data_ptr();
  a.B = (const uint16_t*)B.data_ptr();
  a.C = C.data_ptr();
  a.Cin = ptr_or_null(Cin);
  a.bias = ptr_or_null(bias);
  a.bias_type = bias.has_value() ? (bias->scalar_type() == at::kFloat ? 2 : 1) : 0;
  a.aux_in = (const uint16_t*)ptr_or_null(aux_in);
  a.aux_out = (uint16_t*)ptr_or_null(aux_out);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.lda = (int)lda; a.ldb = (int)ldb; a.ldc = (int)ldc;
  a.sA0 = sA0; a.sA1 = sA1; a.sB0 = sB0; a.sB1 = sB1; a.sC0 = sC0; a.sC1 = sC1;
  a.batch_inner = (int)std::max<int64_t>(1, batch_inner);
  a.alpha = (float)alpha; a.beta = (float)beta;
  a.act = (int)act; a.causal = (int)causal;
  a.ws = ws.has_value() ? ws->data_ptr<float>() : nullptr;
  a.ws_elems = ws.has_value() ? ws->numel() : 0;
  a.tile_cfg = (int)tile_cfg;
  if (alpha_dev.has_value()) {
    TORCH_CHECK(alpha_dev->scalar_type() == at::kFloat && alpha_dev->numel() == 1 && alpha_dev->is_cuda(),
                "alpha_dev must be a 1-element fp32 GPU tensor");
    a.alpha_dev = alpha_dev->data_ptr<float>();
  }
  if (cs_out.has_value()) {  // column sums of C (fp32 [N]) with cs_ws scratch
    TORCH_CHECK(cs_ws.has_value() && cs_out->scalar_type() == at::kFloat && cs_out->numel() >= N &&
                    cs_ws->scalar_type() == at::kFloat && batch == 1,
                "gemm_bf16: cs_out needs fp32 [N] + fp32 cs_ws scratch, batch 1");
    a.cs_out = cs_out->data_ptr<float>();
    a.cs_ws = cs_ws->data_ptr<float>();
    a.cs_ws_elems = cs_ws->numel();
  } else if (cs_ws.has_value()) {  // deferred: partial rows only
    TORCH_CHECK(cs_ws->scalar_type() == at::kFloat && batch == 1, "gemm_bf16: cs_ws needs fp32 scratch, batch 1");
    a.cs_ws = cs_ws->data_ptr<float>();
    a.cs_ws_elems = cs_ws->numel();
  }
  TORCH_CHECK(act >= 0 && act <= 6, "gemm_bf16: act 0..6");
  TORCH_CHECK(!(act == 2 || act == 5) || a.aux_out, "gelu forward needs aux_out");
  TORCH_CHECK(!(act == 3 || act == 4 || act == 6) || a.aux_in, "activation backward needs aux_in");
  int cs_rows = 0;
  check_rc(rtdc_gemm_bf16(&a, a_kmajor, b_kmajor, C.scalar_type() == at::kFloat, (int)batch, cur_stream(),
                          &cs_rows),
           "gemm_bf16");
  return cs_rows;
}

// Independent plain products C_i = A_i . B_i in ONE launch of the 8-wave kernel (gemm_8ph.hip
// gemm8g_kernel): dims = [M, N, K, lda, ldb, ldc] per product.  Layouts / output dtype shared;
// currently the weight-gradient form (both operands MN-major, fp32 C).
static void gemm_bf16_grouped(std::vector<Tensor> A, std::vector<Tensor> B, std::vector<Tensor> C,
                              std::vector<int64_t> dims, bool a_kmajor, bool b_kmajor) {
  const size_t n = A.size();
  TORCH_CHECK(n >= 1 && n <= 10 && B.size() == n && C.size() == n && dims.size() == 6 * n,
              "gemm_bf16_grouped: 1..10 products, 6 dims each");
  std::vector<rtdc::GemmArgs> args(n);
  const bool fp32 = C[0].scalar_type() == at::kFloat;
  for (size_t i = 0; i < n; ++i) {
    check_dev(A[i], "A");
    check_dev(B[i], "B");
    check_dev(C[i], "C");
    TORCH_CHECK(A[i].scalar_type() == at::kBFloat16 && B[i].scalar_type() == at::kBFloat16, "A/B must be bf16");
    TORCH_CHECK((C[i].scalar_type() == at::kFloat) == fp32, "gemm_bf16_grouped: one output dtype");
    const int64_t* d = &dims[6 * i];
    const int64_t M = d[0], N = d[1], K = d[2];
    TORCH_CHECK(K % 64 == 0 && M % 8 == 0 && N % 8 == 0 && d[3] % 8 == 0 && d[4] % 8 == 0 && d[5] % 4 == 0,
                "gemm_bf16_grouped: need K%64==0, M%8==0, N%8==0 and 16-B leading dims");
    // the operands must cover what the kernel reads (MN-major: K rows of ld elements)
    TORCH_CHECK(A[i].numel() >= (a_kmajor ? M * d[3] : K * d[3]) && B[i].numel() >= (b_kmajor ? N * d[4] : K * d[4]) &&
                    C[i].numel() >= M * d[5],
                "gemm_bf16_grouped: operand smaller than its dims");
    rtdc::GemmArgs& a = args[i];
    a = rtdc::GemmArgs{};
    a.A = (const uint16_t*)A[i].data_ptr();
    a.B = (const uint16_t*)B[i].data_ptr();
    a.C = C[i].data_ptr();
    a.M = (int)M; a.N = (int)N; a.K = (int)K;
    a.lda = (int)d[3]; a.ldb = (int)d[4]; a.ldc = (int)d[5];
    a.batch_inner = 1;
    a.alpha = 1.f;
    a.splitk = 1;
    a.tile_cfg = -1;
  }
  check_rc(rtdc_gemm8_grouped(args.data(), (int)n, a_kmajor, b_kmajor, fp32, cur_stream()), "gemm_bf16_grouped");
}

static void gemm_f32(Tensor A, Tensor B, Tensor C, c10::optional<Tensor> Cin, c10::optional<Tensor> bias,
                     c10::optional<Tensor> aux_in, c10::optional<Tensor> aux_out, int64_t M, int64_t N,
                     int64_t K, int64_t sam, int64_t sak, int64_t sbk, int64_t sbn, int64_t ldc, double alpha,
                     double beta, int64_t act, double drop_p, uint64_t drop_seed, uint64_t drop_offset,
                     c10::optional<Tensor> drop_base) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm_f32 needs GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kFloat && B.scalar_type() == at::kFloat && C.scalar_type() == at::kFloat,
              "gemm_f32: fp32 only");
  rtdc::GemmF32Args a{};
  a.A = A.data_ptr<float>();
  a.B = B.data_ptr<float>();
  a.C = C.data_ptr<float>();
  a.Cin = (const float*)ptr_or_null(Cin);
  a.bias = (const float*)ptr_or_null(bias);
  a.aux_in = (const float*)ptr_or_null(aux_in);
  a.aux_out = (float*)ptr_or_null(aux_out);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.sam = sam; a.sak = sak; a.sbk = sbk; a.sbn = sbn;
  a.ldc = (int)ldc;
  a.alpha = (float)alpha; a.beta = (float)beta; a.act = (int)act;
  TORCH_CHECK(drop_p == 0.0 || (act == 1 && drop_p > 0.0 && drop_p < 1.0 && ldc == N),
              "gemm_f32: fused dropout needs act=relu, 0 < p < 1 and a dense output");
  TORCH_CHECK(!drop_base.has_value() || (drop_base->scalar_type() == at::kLong && drop_base->is_cuda()),
              "gemm_f32: drop_base must be an int64 GPU tensor");
  a.drop_p = (float)drop_p;
  a.drop_seed = drop_seed;
  a.drop_offset = drop_offset;
  a.drop_base = drop_base.has_value() ? (const long long*)drop_base->data_ptr<int64_t>() : nullptr;
  check_rc(rtdc_gemm_f32(&a, cur_stream()), "gemm_f32");
}

// ---------------------------------------------------------------------------------- norms
static void layernorm_fwd(Tensor x, Tensor g, Tensor b, Tensor y, Tensor mean, Tensor rstd, double eps) {
  check_dev(x, "x");
  const int D = (int)x.size(-1), M = (int)(x.numel() / D);
  check_rc(rtdc_layernorm_fwd(x.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr<float>(),
                              rstd.data_ptr<float>(), M, D, (float)eps, cur_stream()),
           "layernorm_fwd");
}
static void rmsnorm_fwd(Tensor x, Tensor g, Tensor y, Tensor rstd, double eps) {
  check_dev(x, "x");
  const int D = (int)x.size(-1), M = (int)(x.numel() / D);
  check_rc(rtdc_rmsnorm_fwd(x.data_ptr(), g.data_ptr(), y.data_ptr(), rstd.data_ptr<float>(), M, D, (float)eps,
                            cur_stream()),
           "rmsnorm_fwd");
}
// dxsum (optional, fp32 [D]): column sums of dx, produced by the same kernel
// defer=true: only the partial rows [nz][nblk][D] are written to ws (nz = 2 + has dxsum: dgamma,
// dbeta, colsum(dx)); returns nblk, and the caller reduces them later (colsum_multi).  Else 0.
static int64_t layernorm_bwd(Tensor dy, Tensor x, Tensor g, Tensor mean, Tensor rstd, c10::optional<Tensor> dres,
                             Tensor dx, Tensor ws, Tensor dg, Tensor db, c10::optional<Tensor> dxsum, int64_t nwaves,
                             bool accumulate, bool defer) {
  const int D = (int)x.size(-1), M = (int)(x.numel() / D);
  const int nz = 2 + (dxsum.has_value() ? 1 : 0);
  TORCH_CHECK(ws.numel() >= nz * (nwaves / 4 + 64) * D, "layernorm_bwd workspace too small");
  if (dxsum.has_value()) TORCH_CHECK(dxsum->numel() >= D && dxsum->scalar_type() == at::kFloat, "dxsum: fp32 [D]");
  int nblk = 0;
  check_rc(rtdc_layernorm_bwd(dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr<float>(),
                              rstd.data_ptr<float>(), ptr_or_null(dres), dx.data_ptr(), ws.data_ptr<float>(),
                              dg.data_ptr<float>(), db.data_ptr<float>(), (float*)ptr_or_null(dxsum), M, D,
                              (int)nwaves, accumulate, cur_stream(), defer ? &nblk : nullptr),
           "layernorm_bwd");
  return defer ? nblk : 0;
}
static void rmsnorm_bwd(Tensor dy, Tensor x, Tensor g, Tensor rstd, c10::optional<Tensor> dres, Tensor dx,
                        Tensor ws, Tensor dg, c10::optional<Tensor> dxsum, int64_t nwaves, bool accumulate) {
  const int D = (int)x.size(-1), M = (int)(x.numel() / D);
  const int nz = 1 + (dxsum.has_value() ? 1 : 0);
  TORCH_CHECK(ws.numel() >= nz * (nwaves / 4 + 64) * D, "rmsnorm_bwd workspace too small");
  if (dxsum.has_value()) TORCH_CHECK(dxsum->numel() >= D && dxsum->scalar_type() == at::kFloat, "dxsum: fp32 [D]");
  check_rc(rtdc_rmsnorm_bwd(dy.data_ptr(), x.data_ptr(), g.data_ptr(), rstd.data_ptr<float>(), ptr_or_null(dres),
                            dx.data_ptr(), ws.data_ptr<float>(), dg.data_ptr<float>(), (float*)ptr_or_null(dxsum), M,
                            D, (int)nwaves, accumulate, cur_stream()),
           "rmsnorm_bwd");
}
static void colsum_partial(Tensor X, int64_t M, int64_t N, int64_t ld, Tensor ws, int64_t nblk) {
  TORCH_CHECK(ws.numel() >= nblk * N && ws.scalar_type() == at::kFloat, "colsum_partial workspace too small");
  check_rc(rtdc_colsum_partial(X.data_ptr(), (int)M, (int)N, (int)ld, ws.data_ptr<float>(), (int)nblk,
                               X.scalar_type() == at::kBFloat16, cur_stream()),
           "colsum_partial");
}
// n <= 32 deferred reductions out_j (+)= sum of the W_j partial rows ws_j [W_j][D_j], one launch
static void colsum_multi(std::vector<Tensor> ws, std::vector<Tensor> out, std::vector<int64_t> W,
                         std::vector<int64_t> D, std::vector<int64_t> accumulate) {
  const size_t n = ws.size();
  TORCH_CHECK(n >= 1 && n <= 32 && out.size() == n && W.size() == n && D.size() == n && accumulate.size() == n,
              "colsum_multi: 1..32 jobs");
  std::vector<const float*> wp(n);
  std::vector<float*> op(n);
  std::vector<int> wi(n), di(n), ai(n);
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(ws[i].is_cuda() && ws[i].scalar_type() == at::kFloat && ws[i].numel() >= W[i] * D[i],
                "colsum_multi: fp32 ws [W][D]");
    TORCH_CHECK(out[i].is_cuda() && out[i].scalar_type() == at::kFloat && out[i].numel() >= D[i] &&
                    out[i].is_contiguous(),
                "colsum_multi: fp32 out [D]");
    wp[i] = ws[i].data_ptr<float>();
    op[i] = out[i].data_ptr<float>();
    wi[i] = (int)W[i];
    di[i] = (int)D[i];
    ai[i] = accumulate[i] ? 1 : 0;
  }
  check_rc(rtdc_colsum_multi(wp.data(), op.data(), wi.data(), di.data(), ai.data(), (int)n, cur_stream()),
           "colsum_multi");
}
static void colsum(Tensor X, int64_t M, int64_t N, int64_t ld, Tensor ws, int64_t nblk, Tensor out,
                   bool accumulate) {
  TORCH_CHECK(ws.numel() >= (nblk + 64) * N, "colsum workspace too small");
  check_rc(rtdc_colsum(X.data_ptr(), (int)M, (int)N, (int)ld, ws.data_ptr<float>(), (int)nblk,
                       out.data_ptr<float>(), accumulate, X.scalar_type() == at::kBFloat16, cur_stream()),
           "colsum");
}

// ---------------------------------------------------------------------------------- xent
static void xent(Tensor logits, c10::optional<Tensor> dlogits, c10::optional<Tensor> target,
                 c10::optional<Tensor> loss, c10::optional<Tensor> lse, c10::optional<Tensor> argmax, int64_t M,
                 int64_t V, int64_t ld, double grad_scale, int64_t ignore_index) {
  TORCH_CHECK(logits.is_cuda(), "xent: GPU tensor expected");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat,
              "xent: logits must be fp32 or bf16");
  TORCH_CHECK(logits.is_contiguous() && ld >= V && logits.numel() >= M * ld, "xent: logits [M, ld] contiguous");
  if (dlogits.has_value())
    TORCH_CHECK(dlogits->scalar_type() == logits.scalar_type() && dlogits->is_contiguous() &&
                    dlogits->numel() >= M * ld,
                "xent: dlogits must match logits");
  if (target.has_value())
    TORCH_CHECK(target->scalar_type() == at::kLong && target->is_contiguous() && target->numel() >= M,
                "xent: target must be a contiguous int64 [M] tensor");
  if (loss.has_value())
    TORCH_CHECK(loss->scalar_type() == at::kFloat && loss->is_contiguous() && loss->numel() >= M,
                "xent: loss must be a contiguous fp32 [M] tensor");
  if (lse.has_value()) TORCH_CHECK(lse->scalar_type() == at::kFloat && lse->numel() >= M, "xent: lse fp32 [M]");
  if (argmax.has_value())
    TORCH_CHECK(argmax->scalar_type() == at::kLong && argmax->numel() >= M, "xent: argmax int64 [M]");
  check_rc(rtdc_xent(logits.data_ptr(), ptr_or_null(dlogits), (const int64_t*)ptr_or_null(target),
                     (float*)ptr_or_null(loss), (float*)ptr_or_null(lse), (int64_t*)ptr_or_null(argmax), (int)M,
                     (int)V, (int)ld, (float)grad_scale, (int)ignore_index,
                     logits.scalar_type() == at::kBFloat16, cur_stream()),
           "xent");
}

// ---------------------------------------------------------------------------------- optim
// chunk tables: int64 [n, 3] rows (start, len | decay << 32, state start) - kernels/optim.hip Chunk
static void check_chunks(const Tensor& chunks, int64_t nchunks, const char* op) {
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong && chunks.is_contiguous() && chunks.dim() == 2 &&
                  chunks.size(1) == 3 && chunks.size(0) >= nchunks,
              op, ": chunk table must be a contiguous int64 [n, 3] GPU tensor");
}
static void adamw(Tensor chunks, int64_t nchunks, Tensor p, Tensor g, Tensor m, Tensor v,
                  c10::optional<Tensor> shadow, double lr, double b1, double b2, double eps, double wd, double bc1,
                  double bc2_sqrt, double grad_scale, int64_t skip_ptr) {
  check_chunks(chunks, nchunks, "adamw");
  check_rc(rtdc_adamw(chunks.data_ptr(), (int)nchunks, p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                      v.data_ptr<float>(), ptr_or_null(shadow), (float)lr, (float)b1, (float)b2, (float)eps,
                      (float)wd, (float)bc1, (float)bc2_sqrt, (float)grad_scale, (const int*)(uintptr_t)skip_ptr,
                      cur_stream()),
           "adamw");
}
static void sgd(Tensor chunks, int64_t nchunks, Tensor p, Tensor g, c10::optional<Tensor> buf,
                c10::optional<Tensor> shadow, double lr, double momentum, double dampening, double wd,
                bool nesterov, bool first, double grad_scale, int64_t skip_ptr) {
  check_chunks(chunks, nchunks, "sgd");
  check_rc(rtdc_sgd(chunks.data_ptr(), (int)nchunks, p.data_ptr<float>(), g.data_ptr<float>(),
                    (float*)ptr_or_null(buf), ptr_or_null(shadow), (float)lr, (float)momentum, (float)dampening,
                    (float)wd, nesterov, first, (float)grad_scale, (const int*)(uintptr_t)skip_ptr, cur_stream()),
           "sgd");
}
static void f32_to_bf16(Tensor x, Tensor y) {
  check_rc(rtdc_f32_to_bf16(x.data_ptr<float>(), y.data_ptr(), (long long)x.numel(), cur_stream()), "f32_to_bf16");
}
// dst[i] = src[i]^T for bf16 [R, C] -> [C, R] matrices in one launch; `jobs` is a uint8 device
// buffer of >= bf16_transpose_jobs_bytes() (the job table, uploaded on the current stream)
static void bf16_transpose_multi(std::vector<Tensor> src, std::vector<Tensor> dst, Tensor jobs) {
  TORCH_CHECK(src.size() == dst.size(), "bf16_transpose_multi: src/dst count");
  TORCH_CHECK(jobs.is_cuda() && jobs.numel() >= rtdc_bf16_transpose_jobs_bytes(), "bf16_transpose_multi: jobs buffer");
  std::vector<const void*> s;
  std::vector<void*> d;
  std::vector<int> R, C;
  for (size_t i = 0; i < src.size(); ++i) {
    const Tensor& x = src[i];
    const Tensor& y = dst[i];
    TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.scalar_type() == at::kBFloat16 && x.is_contiguous(),
                "bf16_transpose_multi: contiguous bf16 [R, C] sources");
    TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.scalar_type() == at::kBFloat16 && y.is_contiguous() &&
                    y.size(0) == x.size(1) && y.size(1) == x.size(0),
                "bf16_transpose_multi: contiguous bf16 [C, R] destinations");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(y.data_ptr()) & 15) == 0,
                "bf16_transpose_multi: 16-B aligned operands");
    s.push_back(x.data_ptr());
    d.push_back(y.data_ptr());
    R.push_back((int)x.size(0));
    C.push_back((int)x.size(1));
  }
  check_rc(rtdc_bf16_transpose_multi(s.data(), d.data(), R.data(), C.data(), (int)s.size(), jobs.data_ptr(),
                                     cur_stream()),
           "bf16_transpose_multi");
}
static void f32_to_bf16_t(Tensor x, Tensor y) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.scalar_type() == at::kFloat && x.is_contiguous(),
              "f32_to_bf16_t: contiguous fp32 [R, C]");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.dim() == 2 &&
                  y.size(0) == x.size(1) && y.size(1) == x.size(0),
              "f32_to_bf16_t: contiguous bf16 [C, R]");
  check_rc(rtdc_f32_to_bf16_t(x.data_ptr<float>(), y.data_ptr(), (int)x.size(0), (int)x.size(1), cur_stream()),
           "f32_to_bf16_t");
}
static void sumsq(Tensor chunks, int64_t nchunks, Tensor g, Tensor partial) {
  check_chunks(chunks, nchunks, "sumsq");
  check_rc(rtdc_sumsq(chunks.data_ptr(), (int)nchunks, g.data_ptr<float>(), partial.data_ptr<float>(), cur_stream()),
           "sumsq");
}

// ---------------------------------------------------------------------------------- attention softmax
static void softmax_fwd(Tensor S, Tensor P, c10::optional<Tensor> lse, int64_t rows, int64_t T, bool causal) {
  check_rc(rtdc_softmax_fwd(S.data_ptr(), P.data_ptr(), (float*)ptr_or_null(lse), rows, (int)T, causal, cur_stream()),
           "softmax_fwd");
}
static void softmax_bwd(Tensor P, Tensor dP, Tensor dS, int64_t rows, int64_t T, bool causal) {
  check_rc(rtdc_softmax_bwd(P.data_ptr(), dP.data_ptr(), dS.data_ptr(), rows, (int)T, causal, cur_stream()),
           "softmax_bwd");
}

// ---------------------------------------------------------------------------------- embedding / dropout
static void embed_fwd(Tensor idx, Tensor wte, c10::optional<Tensor> wpe, Tensor out, int64_t T) {
  const int D = (int)wte.size(1);
  check_rc(rtdc_embed_fwd(idx.data_ptr<int64_t>(), wte.data_ptr(), ptr_or_null(wpe), out.data_ptr(),
                          (int)idx.numel(), (int)T, D, cur_stream()),
           "embed_fwd");
}
// stable sort of token ids (< 2^nbits): sorted ids + original positions, one workgroup
static void sort_ids(Tensor ids, Tensor sorted, Tensor perm, Tensor ws, int64_t nbits) {
  const int64_t n = ids.numel();
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "sort_ids: ids must be contiguous int64 on the GPU");
  TORCH_CHECK(sorted.numel() == n && perm.numel() == n && sorted.scalar_type() == at::kLong &&
                  perm.scalar_type() == at::kLong && sorted.is_contiguous() && perm.is_contiguous(),
              "sort_ids: outputs must be contiguous int64 of ids.numel()");
  TORCH_CHECK(ws.numel() * ws.element_size() >= 16 * n && ws.is_contiguous(), "sort_ids: workspace needs 16 B per id");
  TORCH_CHECK(n < (1LL << 31), "sort_ids: too many ids");
  check_rc(rtdc_sort_ids(ids.data_ptr<int64_t>(), (int)n, (int)nbits, (uint32_t*)ws.data_ptr(),
                         sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), cur_stream()),
           "sort_ids");
}
// inputs/targets [B, T] int64 of the synthetic sequences ids[B] (workloads.SyntheticTokens)
static void synth_tokens(Tensor ids, Tensor inp, Tensor tgt, int64_t vocab, int64_t seed_add) {
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.dim() == 1,
              "synth_tokens: ids must be a contiguous 1-D int64 GPU tensor");
  const int64_t B = ids.numel();
  TORCH_CHECK(inp.dim() == 2 && inp.size(0) == B && tgt.sizes() == inp.sizes() && inp.is_contiguous() &&
                  tgt.is_contiguous() && inp.scalar_type() == at::kLong && tgt.scalar_type() == at::kLong,
              "synth_tokens: inp/tgt must be contiguous int64 [B, T]");
  check_rc(rtdc_synth_tokens(ids.data_ptr<int64_t>(), (int)B, (int)inp.size(1), (long long)vocab,
                             (unsigned long long)seed_add, inp.data_ptr<int64_t>(), tgt.data_ptr<int64_t>(),
                             cur_stream()),
           "synth_tokens");
}
// sidx / perm: stably sorted token ids and their original positions (deterministic backward)
static void fill_f32(Tensor x, double v) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "fill_f32: contiguous fp32 CUDA tensor");
  if (x.numel() == 0) return;
  TORCH_CHECK(((uintptr_t)x.data_ptr() & 15) == 0, "fill_f32: 16-B aligned tensor");
  check_rc(rtdc_fill_f32(x.data_ptr<float>(), (long long)x.numel(), (float)v, cur_stream()), "fill_f32");
}
static void embed_bwd(Tensor sidx, Tensor perm, Tensor dout, Tensor dwte, c10::optional<Tensor> dwpe, int64_t B,
                      int64_t T, bool accumulate_wpe, bool accumulate_wte) {
  const int D = (int)dwte.size(1);
  TORCH_CHECK(sidx.is_contiguous() && perm.is_contiguous() && sidx.numel() == B * T, "embed_bwd: bad sort arrays");
  check_rc(rtdc_embed_bwd(sidx.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dout.data_ptr(), dwte.data_ptr<float>(),
                          (float*)ptr_or_null(dwpe), (int)B, (int)T, D, accumulate_wpe, accumulate_wte, cur_stream()),
           "embed_bwd");
}
static void dropout(Tensor x, Tensor y, double p, uint64_t seed, uint64_t offset, c10::optional<Tensor> off_dev) {
  TORCH_CHECK(!off_dev.has_value() || (off_dev->scalar_type() == at::kLong && off_dev->is_cuda()),
              "dropout: off_dev must be an int64 GPU tensor");
  check_rc(rtdc_dropout(x.data_ptr(), y.data_ptr(), (long long)x.numel(), (float)p, seed, offset,
                        off_dev.has_value() ? (const long long*)off_dev->data_ptr<int64_t>() : nullptr,
                        x.scalar_type() == at::kBFloat16, cur_stream()),
           "dropout");
}
static void relu_dropout(Tensor h, c10::optional<Tensor> y, c10::optional<Tensor> dy, c10::optional<Tensor> dx,
                         double p, uint64_t seed, uint64_t offset, int64_t backward) {
  check_rc(rtdc_relu_dropout(h.data_ptr(), ptr_or_null(y), ptr_or_null(dy), ptr_or_null(dx), (long long)h.numel(),
                             (float)p, seed, offset, (int)backward, h.scalar_type() == at::kBFloat16, cur_stream()),
           "relu_dropout");
}

// ---------------------------------------------------------------------------------- flash attention
static void flash_fwd(Tensor qkv, Tensor out, Tensor lse, int64_t B, int64_t T, int64_t H, int64_t Hkv, int64_t Dh,
                      double scale) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.is_contiguous() && out.is_contiguous(), "flash_fwd: contiguous tensors expected");
  check_rc(rtdc_flash_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), (int)B, (int)T, (int)H, (int)Hkv,
                          (int)Dh, (float)scale, cur_stream()),
           "flash_fwd");
}
// cs_ws (optional fp32 [B*T/16][W], W = (H + 2 Hkv) Dh): per 16-row group column sums of dqkv
static void flash_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, Tensor delta, Tensor dqkv, int64_t B, int64_t T,
                      int64_t H, int64_t Hkv, int64_t Dh, double scale, c10::optional<Tensor> cs_ws,
                      c10::optional<Tensor> part, int64_t qs, int64_t which, bool delta_ready) {
  TORCH_CHECK(dout.is_contiguous() && dqkv.is_contiguous(), "flash_bwd: contiguous tensors expected");
  TORCH_CHECK(qs >= 1 && (H / Hkv) % qs == 0, "flash_bwd: qs must divide the GQA group size");
  if (qs > 1)
    TORCH_CHECK(part.has_value() && part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() >= qs * B * T * Hkv * 2 * Dh,
                "flash_bwd: part fp32 [qs][B*T][Hkv][2*Dh] workspace");
  if (cs_ws.has_value())
    TORCH_CHECK(cs_ws->is_cuda() && cs_ws->scalar_type() == at::kFloat && cs_ws->is_contiguous() &&
                    cs_ws->numel() >= B * T / 16 * (H + 2 * Hkv) * Dh,
                "flash_bwd: cs_ws fp32 [B*T/16][W]");
  check_rc(rtdc_flash_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                          delta.data_ptr<float>(), dqkv.data_ptr(), (int)B, (int)T, (int)H, (int)Hkv, (int)Dh,
                          (float)scale, cs_ws.has_value() ? cs_ws->data_ptr<float>() : nullptr,
                          qs > 1 ? part->data_ptr<float>() : nullptr, (int)qs, (int)which, delta_ready ? 1 : 0,
                          cur_stream()),
           "flash_bwd");
}
// delta[B*H][T] = rowsum(dO * O) on its own (then flash_bwd(..., which=1|2, delta_ready=True))
static void flash_delta(Tensor out, Tensor dout, Tensor delta, int64_t B, int64_t T, int64_t H, int64_t Dh) {
  TORCH_CHECK(out.is_contiguous() && dout.is_contiguous() && delta.is_contiguous() &&
                  delta.scalar_type() == at::kFloat && delta.numel() >= B * H * T,
              "flash_delta: contiguous out / dout and fp32 delta [B*H][T] expected");
  check_rc(rtdc_flash_delta(out.data_ptr(), dout.data_ptr(), delta.data_ptr<float>(), (int)B, (int)T, (int)H, (int)Dh,
                            cur_stream()),
           "flash_delta");
}

// ---------------------------------------------------------------------------------- llama ops
static void rope(Tensor x, Tensor y, Tensor cosb, Tensor sinb, int64_t T, int64_t nrot_heads, int64_t ntot_heads,
                 int64_t Dh, bool inverse) {
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous(), "rope: contiguous tensors expected");
  const int64_t ntok = x.numel() / (ntot_heads * Dh);
  check_rc(rtdc_rope(x.data_ptr(), y.data_ptr(), cosb.data_ptr<float>(), sinb.data_ptr<float>(), (int)ntok, (int)T,
                     (int)nrot_heads, (int)ntot_heads, (int)Dh, inverse, cur_stream()),
           "rope");
}
static void swiglu_fwd(Tensor gu, Tensor h) {
  const int64_t F = h.size(-1), M = h.numel() / F;
  check_rc(rtdc_swiglu_fwd(gu.data_ptr(), h.data_ptr(), M, (int)F, cur_stream()), "swiglu_fwd");
}
static void swiglu_bwd(Tensor gu, Tensor dh, Tensor dgu) {
  const int64_t F = dh.size(-1), M = dh.numel() / F;
  check_rc(rtdc_swiglu_bwd(gu.data_ptr(), dh.data_ptr(), dgu.data_ptr(), M, (int)F, cur_stream()), "swiglu_bwd");
}

// ---------------------------------------------------------------------------------- conv / batchnorm / pooling
// Implicit-GEMM convolution products (gemm_bf16.hip, rtdc_conv_gemm):
//   mode 1: C[npix, N] bf16 = im2col(X) . other[N, K]^T          (other K-major, ld = ld_other)
//   mode 2: C[M, N]    fp32 = other[K, M]^T . im2col(X)           (other = dY, MN-major, ld = ld_other)
// X is NHWC [B, H, W, Cx]; the window is KH x KW (K = KH*KW*Cx in mode 1, N in mode 2).
// stats_mean/stats_m2 (mode 1, optional): fused BatchNorm statistics per output row tile,
// [ceil(M/128)][N] fp32; returns the rows per statistics tile (128 or 256).
static int64_t conv_gemm_impl(Tensor X, Tensor other, Tensor C, int64_t mode, int64_t M, int64_t N, int64_t K,
                              int64_t ld_other, int64_t Ho, int64_t Wo, int64_t KW, int64_t stride, int64_t pad,
                              c10::optional<Tensor> ws, c10::optional<Tensor> stats_mean,
                              c10::optional<Tensor> stats_m2, c10::optional<Tensor> accumulate,
                              const std::vector<Tensor>* bnb) {
  check_dev(X, "X");
  check_dev(other, "other");
  TORCH_CHECK(X.is_contiguous() && X.dim() == 4 && X.scalar_type() == at::kBFloat16, "conv_gemm: X must be NHWC bf16");
  TORCH_CHECK(other.scalar_type() == at::kBFloat16 && C.is_contiguous(), "conv_gemm: bad operands");
  const int64_t npix = X.size(0) * Ho * Wo;
  if (mode == 1) {
    TORCH_CHECK(C.scalar_type() == at::kBFloat16 && C.size(0) == npix && C.size(1) == N && M == npix, "conv_gemm: C");
  } else {
    TORCH_CHECK(C.scalar_type() == at::kFloat && C.size(0) == M && C.size(1) == N && K >= npix, "conv_gemm: C");
    TORCH_CHECK(other.size(0) >= K, "conv_gemm: dY must have K (padded) rows");
  }
  rtdc::GemmArgs a{};
  a.A = (const uint16_t*)(mode == 1 ? X.data_ptr() : other.data_ptr());
  a.B = (const uint16_t*)(mode == 1 ? other.data_ptr() : X.data_ptr());
  a.C = C.data_ptr();
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.lda = mode == 1 ? 0 : (int)ld_other;
  a.ldb = mode == 1 ? (int)ld_other : 0;
  a.ldc = (int)N;
  a.batch_inner = 1;
  a.alpha = 1.f;
  a.beta = 0.f;
  a.tile_cfg = -1;
  if (ws.has_value()) {
    a.ws = ws->data_ptr<float>();
    a.ws_elems = ws->numel();
  }
  a.cv_H = (int)X.size(1); a.cv_W = (int)X.size(2); a.cv_C = (int)X.size(3);
  a.cv_Ho = (int)Ho; a.cv_Wo = (int)Wo; a.cv_KW = (int)KW; a.cv_stride = (int)stride; a.cv_pad = (int)pad;
  a.cv_npix = (int)npix;
  const int64_t bm = N <= 64 ? 256 : 128;
  if (stats_mean.has_value()) {
    TORCH_CHECK(mode == 1 && stats_m2.has_value(), "conv_gemm: statistics need mode 1 and both buffers");
    TORCH_CHECK(stats_mean->numel() >= ((M + bm - 1) / bm) * N && stats_m2->numel() >= ((M + bm - 1) / bm) * N,
                "conv_gemm: statistics buffers too small");
    a.stats_mean = stats_mean->data_ptr<float>();
    a.stats_m2 = stats_m2->data_ptr<float>();
  }
  if (accumulate.has_value()) {  // C = conv(...) + accumulate (mode 1: a residual-path gradient)
    TORCH_CHECK(mode == 1 && accumulate->scalar_type() == C.scalar_type() && accumulate->is_contiguous() &&
                    accumulate->numel() == C.numel(),
                "conv_gemm: accumulate must match C (mode 1)");
    a.Cin = accumulate->data_ptr();
    a.beta = 1.f;
  }
  if (bnb) {  // [x, mean, rstd, gamma, beta (, y)]: BatchNorm-backward statistics into stats_mean / stats_m2
    TORCH_CHECK(mode == 1 && (bnb->size() == 5 || bnb->size() == 6) && stats_mean.has_value() && stats_m2.has_value(),
                "conv_gemm_bnb: mode 1, [x, mean, rstd, gamma, beta (, y)] and both statistics buffers");
    const Tensor& x = (*bnb)[0];
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.numel() == C.numel(),
                "conv_gemm_bnb: x must match C");
    for (int i = 1; i < 5; ++i)
      TORCH_CHECK((*bnb)[i].is_cuda() && (*bnb)[i].scalar_type() == at::kFloat && (*bnb)[i].numel() >= N,
                  "conv_gemm_bnb: fp32 [N] BatchNorm parameters");
    a.bnb_x = (const uint16_t*)x.data_ptr();
    a.bnb_mean = (*bnb)[1].data_ptr<float>();
    a.bnb_rstd = (*bnb)[2].data_ptr<float>();
    a.bnb_gamma = (*bnb)[3].data_ptr<float>();
    a.bnb_beta = (*bnb)[4].data_ptr<float>();
    if (bnb->size() == 6) {  // ReLU mask from the BN + residual output y
      const Tensor& y = (*bnb)[5];
      TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.numel() == C.numel(),
                  "conv_gemm_bnb: y must match C");
      a.bnb_y = (const uint16_t*)y.data_ptr();
    }
  }
  check_rc(rtdc_conv_gemm(&a, (int)mode, cur_stream()), "conv_gemm");
  return bm;
}
static int64_t conv_gemm(Tensor X, Tensor other, Tensor C, int64_t mode, int64_t M, int64_t N, int64_t K,
                         int64_t ld_other, int64_t Ho, int64_t Wo, int64_t KW, int64_t stride, int64_t pad,
                         c10::optional<Tensor> ws, c10::optional<Tensor> stats_mean, c10::optional<Tensor> stats_m2,
                         c10::optional<Tensor> accumulate) {
  return conv_gemm_impl(X, other, C, mode, M, N, K, ld_other, Ho, Wo, KW, stride, pad, ws, stats_mean, stats_m2,
                        accumulate, nullptr);
}
// stride-1 dgrad whose output is the gradient at relu(BN(x)): also the BatchNorm-backward
// partial sums (sum g, sum g*xhat) per row tile - returns the tile height (rows per partial)
static int64_t conv_gemm_bnb(Tensor X, Tensor other, Tensor C, int64_t M, int64_t N, int64_t K, int64_t ld_other,
                             int64_t Ho, int64_t Wo, int64_t KW, int64_t pad, Tensor psum, Tensor psumx,
                             c10::optional<Tensor> accumulate, std::vector<Tensor> bnb) {
  return conv_gemm_impl(X, other, C, 1, M, N, K, ld_other, Ho, Wo, KW, 1, pad, c10::nullopt, psum, psumx, accumulate,
                        &bnb);
}

// x: NHWC bf16 [B,H,W,C]; cols: [B*Ho*Wo, Kp] with K = KH*KW*C real columns (rest zero).
static void im2col(Tensor x, Tensor cols, int64_t Ho, int64_t Wo, int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  TORCH_CHECK(x.is_contiguous() && cols.is_contiguous() && x.dim() == 4, "im2col: contiguous NHWC expected");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), K = KH * KW * C, Kp = cols.size(1);
  TORCH_CHECK(cols.size(0) == B * Ho * Wo && Kp >= K, "im2col: bad cols shape");
  check_rc(rtdc_im2col(x.data_ptr(), cols.data_ptr(), (int)B, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)KH,
                       (int)KW, (int)stride, (int)pad, (int)K, (int)Kp, cur_stream()),
           "im2col");
}
static void col2im(Tensor dcols, Tensor dx, int64_t Ho, int64_t Wo, int64_t KH, int64_t KW, int64_t stride,
                   int64_t pad, c10::optional<Tensor> addend) {
  TORCH_CHECK(dx.is_contiguous() && dcols.is_contiguous() && dx.dim() == 4, "col2im: contiguous NHWC expected");
  const int64_t B = dx.size(0), H = dx.size(1), W = dx.size(2), C = dx.size(3), K = KH * KW * C, Kp = dcols.size(1);
  TORCH_CHECK(dcols.size(0) == B * Ho * Wo && Kp >= K, "col2im: bad cols shape");
  TORCH_CHECK(dcols.scalar_type() == at::kBFloat16 && dx.scalar_type() == at::kBFloat16, "col2im: bf16 expected");
  const void* add = nullptr;
  if (addend.has_value()) {
    TORCH_CHECK(addend->scalar_type() == at::kBFloat16 && addend->is_contiguous() && addend->numel() == dx.numel(),
                "col2im: addend must be a contiguous bf16 tensor shaped like dx");
    add = addend->data_ptr();
  }
  check_rc(rtdc_col2im(dcols.data_ptr(), dx.data_ptr(), add, (int)B, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)KH,
                       (int)KW, (int)stride, (int)pad, (int)K, (int)Kp, cur_stream()),
           "col2im");
}
static void bn_fwd(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> y, Tensor mean, Tensor rstd,
                   Tensor gamma, Tensor beta,
                   c10::optional<Tensor> running_mean, c10::optional<Tensor> running_var, double eps, double momentum,
                   bool training, bool relu, Tensor ws, int64_t nblk, c10::optional<Tensor> pmean,
                   c10::optional<Tensor> pm2, int64_t p_R, c10::optional<Tensor> num_batches_tracked) {
  if (num_batches_tracked.has_value())
    TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong && num_batches_tracked->is_cuda() &&
                    num_batches_tracked->numel() == 1,
                "bn_fwd: num_batches_tracked must be a 1-element int64 GPU tensor");
  const int64_t C = x.size(-1), N = x.numel() / C;
  TORCH_CHECK(x.is_contiguous() && (!y.has_value() || y->is_contiguous()), "bn_fwd: contiguous tensors expected");
  TORCH_CHECK(!training || ws.numel() >= 2 * nblk * C, "bn_fwd: workspace too small");
  check_rc(rtdc_bn_fwd(x.data_ptr(), ptr_or_null(res), ptr_or_null(y), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       gamma.data_ptr<float>(), beta.data_ptr<float>(),
                       running_mean.has_value() ? running_mean->data_ptr<float>() : nullptr,
                       running_var.has_value() ? running_var->data_ptr<float>() : nullptr, N, (int)C, (float)eps,
                       (float)momentum, training, relu, ws.data_ptr<float>(), (int)nblk,
                       pmean.has_value() ? pmean->data_ptr<float>() : nullptr,
                       pm2.has_value() ? pm2->data_ptr<float>() : nullptr,
                       pmean.has_value() ? (int)pmean->size(0) : 0, (int)p_R,
                       num_batches_tracked.has_value() ? (long long*)num_batches_tracked->data_ptr<int64_t>() : nullptr,
                       cur_stream()),
           "bn_fwd");
}
// W'[c][kh'][kw'][co] = W[co][KH-1-kh'][KW-1-kw'][c] (stride-1 conv dgrad operand), bf16
static void conv_w_flip_t(Tensor w, Tensor out, int64_t KH, int64_t KW) {
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16 && w.is_contiguous() &&
                  out.is_contiguous() && w.numel() == out.numel() && w.dim() == 2,
              "conv_w_flip_t: contiguous bf16 [Cout, KH*KW*C] -> [C, KH*KW*Cout]");
  const int64_t Cout = w.size(0), C = w.size(1) / (KH * KW);
  TORCH_CHECK(C * KH * KW == w.size(1), "conv_w_flip_t: bad kernel size");
  check_rc(rtdc_conv_w_flip_t(w.data_ptr(), out.data_ptr(), (int)Cout, (int)KH, (int)KW, (int)C, cur_stream()),
           "conv_w_flip_t");
}
// relu: 0 none, 1 ReLU mask from y (> 0), 2 ReLU mask recomputed from x with gamma / beta (the
// forward had no residual; y is not read)
// ResNet stem as a space-to-depth convolution (cnn.hip): NCHW fp32 image -> [B, H/2, W/2, 16]
// bf16; channels-last bf16 7x7x3 weight [Cout, 147] -> [Cout, 256]; gradient [Cout, 256] fp32 ->
// [Cout, 147] fp32
static void stem_s2d(Tensor x, Tensor y) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4 && x.size(1) == 3,
              "stem_s2d: contiguous fp32 NCHW 3-channel images");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.dim() == 4 && y.size(0) == x.size(0) &&
                  y.size(1) * 2 == x.size(2) && y.size(2) * 2 == x.size(3) && y.size(3) == 16,
              "stem_s2d: y must be [B, H/2, W/2, 16] bf16");
  check_rc(rtdc_stem_s2d(x.data_ptr<float>(), y.data_ptr(), (int)x.size(0), (int)x.size(2), (int)x.size(3),
                         cur_stream()),
           "stem_s2d");
}
static void stem_w_s2d(Tensor w, Tensor wp) {
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() == w.size(0) * 147 &&
                  wp.scalar_type() == at::kBFloat16 && wp.is_contiguous() && wp.numel() == w.size(0) * 256,
              "stem_w_s2d: bf16 [Cout, 7*7*3] -> bf16 [Cout, 256]");
  check_rc(rtdc_stem_w_s2d(w.data_ptr(), wp.data_ptr(), (int)w.size(0), cur_stream()), "stem_w_s2d");
}
static void stem_dw_s2d(Tensor dwp, Tensor dw) {
  TORCH_CHECK(dwp.scalar_type() == at::kFloat && dwp.is_contiguous() && dw.scalar_type() == at::kFloat &&
                  dw.is_contiguous() && dwp.numel() == dwp.size(0) * 256 && dw.numel() == dwp.size(0) * 147,
              "stem_dw_s2d: fp32 [Cout, 256] -> fp32 [Cout, 147]");
  check_rc(rtdc_stem_dw_s2d(dwp.data_ptr<float>(), dw.data_ptr<float>(), (int)dwp.size(0), cur_stream()),
           "stem_dw_s2d");
}
// y [B,Ho,Wo,C] = maxpool(relu(BN(x))) with mean / rstd from bn_fwd (y = None), arg = argmax tap
static void bn_relu_maxpool(Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor beta, Tensor y, Tensor arg,
                            int64_t K, int64_t s, int64_t p) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.is_contiguous() && y.is_contiguous() && arg.is_contiguous() &&
                  x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 &&
                  arg.scalar_type() == at::kByte && arg.sizes() == y.sizes(),
              "bn_relu_maxpool: contiguous bf16 NHWC x / y, uint8 arg shaped like y");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && rstd.scalar_type() == at::kFloat && gamma.scalar_type() == at::kFloat &&
                  beta.scalar_type() == at::kFloat && mean.numel() == x.size(3) && gamma.numel() == x.size(3),
              "bn_relu_maxpool: fp32 per-channel statistics / affine");
  check_rc(rtdc_bn_relu_maxpool(x.data_ptr(), y.data_ptr(), arg.data_ptr(), mean.data_ptr<float>(),
                                rstd.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), (int)x.size(0),
                                (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)y.size(1), (int)y.size(2), (int)K,
                                (int)s, (int)p, cur_stream()),
           "bn_relu_maxpool");
}
static void bn_bwd(Tensor dy, Tensor y, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, c10::optional<Tensor> beta,
                   Tensor dx, c10::optional<Tensor> dres, Tensor dgamma, Tensor dbeta, int64_t relu, Tensor ws,
                   int64_t nblk, c10::optional<Tensor> psum, c10::optional<Tensor> psumx) {
  const int64_t C = x.size(-1), N = x.numel() / C;
  int64_t p_nblk = 0;
  if (psum.has_value()) {  // [p_nblk][C] partials of (sum g, sum g*xhat) from dy's producer
    TORCH_CHECK(psumx.has_value() && psum->scalar_type() == at::kFloat && psumx->scalar_type() == at::kFloat &&
                    psum->dim() == 2 && psum->size(1) == C && psumx->sizes() == psum->sizes() &&
                    psum->is_contiguous() && psumx->is_contiguous(),
                "bn_bwd: psum / psumx fp32 [nblk][C]");
    p_nblk = psum->size(0);
  }
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dx.is_contiguous(), "bn_bwd: contiguous tensors expected");
  TORCH_CHECK(ws.numel() >= 2 * nblk * C, "bn_bwd: workspace too small");
  TORCH_CHECK(relu >= 0 && relu <= 2, "bn_bwd: relu mode 0/1/2");
  TORCH_CHECK(relu != 2 || (beta.has_value() && beta->scalar_type() == at::kFloat && beta->numel() == C),
              "bn_bwd: relu mode 2 needs the fp32 beta");
  check_rc(rtdc_bn_bwd(dy.data_ptr(), y.data_ptr(), x.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       gamma.data_ptr<float>(), relu == 2 ? beta->data_ptr<float>() : nullptr, dx.data_ptr(),
                       ptr_or_null(dres), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), N, (int)C, (int)relu,
                       ws.data_ptr<float>(), (int)nblk, psum.has_value() ? psum->data_ptr<float>() : nullptr,
                       psumx.has_value() ? psumx->data_ptr<float>() : nullptr, (int)p_nblk, cur_stream()),
           "bn_bwd");
}
// mean cross-entropy from per-row losses: out[0] = loss, out[1] = divisor (device count of
// non-ignored targets, or fixed_n when target is None)
static void xent_finalize(Tensor loss, c10::optional<Tensor> target, double fixed_n, Tensor out) {
  check_dev(loss, "loss");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.is_contiguous() && out.scalar_type() == at::kFloat &&
                  out.numel() >= 2 && out.is_contiguous(),
              "xent_finalize: fp32 loss rows / fp32 out[2]");
  const int64_t* t = nullptr;
  if (target.has_value()) {
    TORCH_CHECK(target->scalar_type() == at::kLong && target->is_contiguous() && target->numel() == loss.numel(),
                "xent_finalize: int64 target per row");
    t = target->data_ptr<int64_t>();
  }
  check_rc(rtdc_xent_finalize(loss.data_ptr<float>(), t, (int)loss.numel(), (float)fixed_n, -100,
                              out.data_ptr<float>(), cur_stream()),
           "xent_finalize");
}
static void xent_alpha(Tensor g, Tensor den, Tensor out) {
  TORCH_CHECK(g.scalar_type() == at::kFloat && den.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat,
              "xent_alpha: fp32 scalars");
  check_rc(rtdc_xent_alpha(g.data_ptr<float>(), den.data_ptr<float>(), out.data_ptr<float>(), cur_stream()),
           "xent_alpha");
}
static void scale_dev(Tensor x, Tensor y, Tensor g, Tensor den) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel() && x.scalar_type() == y.scalar_type() &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "scale_dev: matching contiguous bf16/fp32 tensors");
  TORCH_CHECK(g.scalar_type() == at::kFloat && den.scalar_type() == at::kFloat, "scale_dev: fp32 scalars");
  check_rc(rtdc_scale_dev(x.data_ptr(), y.data_ptr(), x.numel(), x.scalar_type() == at::kBFloat16 ? 1 : 0,
                          g.data_ptr<float>(), den.data_ptr<float>(), cur_stream()),
           "scale_dev");
}
static void nchw_to_nhwc_bf16(Tensor x, Tensor y) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4, "nchw_to_nhwc_bf16: contiguous NCHW fp32");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.numel() == x.numel(), "nchw_to_nhwc_bf16: bf16 out");
  check_rc(rtdc_nchw_to_nhwc_bf16(x.data_ptr<float>(), y.data_ptr(), (int)x.size(0), (int)x.size(1),
                                  x.size(2) * x.size(3), cur_stream()),
           "nchw_to_nhwc_bf16");
}
// rows x row_bytes from src (pitch src_pitch bytes) to dst (pitch dst_pitch) on the current
// stream: a DMA-engine copy for padded-operand staging (no ATen kernel)
static void copy2d(Tensor dst, Tensor src, int64_t rows, int64_t row_bytes, int64_t dst_pitch, int64_t src_pitch) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda(), "copy2d: device tensors");
  TORCH_CHECK(row_bytes <= dst_pitch && row_bytes <= src_pitch && rows >= 0, "copy2d: bad geometry");
  TORCH_CHECK((rows - 1) * dst_pitch + row_bytes <= (int64_t)(dst.numel() * dst.element_size()) &&
                  (rows - 1) * src_pitch + row_bytes <= (int64_t)(src.numel() * src.element_size()),
              "copy2d: out of bounds");
  if (rows == 0) return;
  TORCH_CHECK(hipMemcpy2DAsync(dst.data_ptr(), (size_t)dst_pitch, src.data_ptr(), (size_t)src_pitch, (size_t)row_bytes,
                               (size_t)rows, hipMemcpyDeviceToDevice, cur_stream()) == hipSuccess,
              "hipMemcpy2DAsync");
}

static void maxpool_fwd(Tensor x, Tensor y, Tensor arg, int64_t K, int64_t s, int64_t p) {
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && arg.scalar_type() == torch::kUInt8, "maxpool_fwd: bad args");
  check_rc(rtdc_maxpool(x.data_ptr(), y.data_ptr(), arg.data_ptr(), nullptr, nullptr, (int)x.size(0), (int)x.size(1),
                        (int)x.size(2), (int)x.size(3), (int)y.size(1), (int)y.size(2), (int)K, (int)s, (int)p, 0,
                        cur_stream()),
           "maxpool_fwd");
}
// ResNet stem: maxpool3s2(relu(BN(x))) backward in two gather passes; False = shape unsupported
static bool pool_bn_bwd(Tensor dy, Tensor arg, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor beta, Tensor dx,
                        Tensor dgamma, Tensor dbeta, Tensor ws, int64_t nblk) {
  TORCH_CHECK(dy.is_contiguous() && arg.is_contiguous() && x.is_contiguous() && dx.is_contiguous() && x.dim() == 4 &&
                  dy.dim() == 4,
              "pool_bn_bwd: contiguous NHWC tensors expected");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16 && arg.scalar_type() == at::kByte &&
                  gamma.scalar_type() == at::kFloat && beta.scalar_type() == at::kFloat,
              "pool_bn_bwd: bf16 activations, uint8 argmax, fp32 parameters");
  const int C = (int)x.size(3);
  TORCH_CHECK(ws.numel() >= 2 * nblk * C && dgamma.numel() >= C && dbeta.numel() >= C, "pool_bn_bwd: buffers too small");
  const int rc = rtdc_pool_bn_bwd(dy.data_ptr(), arg.data_ptr(), x.data_ptr(), mean.data_ptr<float>(),
                                  rstd.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), dx.data_ptr(),
                                  dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), ws.data_ptr<float>(), (int)nblk,
                                  (int)x.size(0), (int)x.size(1), (int)x.size(2), C, (int)dy.size(1), (int)dy.size(2),
                                  cur_stream());
  if (rc == 1) return false;
  check_rc(rc, "pool_bn_bwd");
  return true;
}
static void maxpool_bwd(Tensor dy, Tensor arg, Tensor dx, int64_t K, int64_t s, int64_t p) {
  TORCH_CHECK(dy.is_contiguous() && dx.is_contiguous(), "maxpool_bwd: contiguous tensors expected");
  check_rc(rtdc_maxpool(nullptr, nullptr, arg.data_ptr(), dy.data_ptr(), dx.data_ptr(), (int)dx.size(0),
                        (int)dx.size(1), (int)dx.size(2), (int)dx.size(3), (int)dy.size(1), (int)dy.size(2), (int)K,
                        (int)s, (int)p, 1, cur_stream()),
           "maxpool_bwd");
}
// x [B, HW, C] <-> y [B, C]
static void avgpool(Tensor x, Tensor y, bool backward) {
  const int64_t B = backward ? y.size(0) : x.size(0), C = backward ? y.size(-1) : x.size(-1);
  const int64_t HW = (backward ? y.numel() : x.numel()) / (B * C);
  check_rc(rtdc_avgpool(x.data_ptr(), y.data_ptr(), (int)B, (int)HW, (int)C, backward, cur_stream()), "avgpool");
}

// ---------------------------------------------------------------------------------- checkpoint engine
using rtdc_ckpt::Engine;
using rtdc_ckpt::FileJob;
using rtdc_ckpt::Record;

// record tuple: (name, data: bytes|None, ptr: int, nbytes: int, on_device: bool)
static std::vector<Record> to_records(const py::list& recs) {
  std::vector<Record> out;
  for (auto item : recs) {
    auto t = item.cast<py::tuple>();
    Record r;
    r.name = t[0].cast<std::string>();
    if (!t[1].is_none()) {
      r.inline_data = t[1].cast<std::string>();
    } else {
      r.src = reinterpret_cast<const char*>(t[2].cast<uintptr_t>());
      r.nbytes = t[3].cast<uint64_t>();
      r.on_device = t[4].cast<bool>();
    }
    out.push_back(std::move(r));
  }
  return out;
}

// archive tuple: (raw: bool, records: list)
static std::vector<rtdc_ckpt::Archive> to_archives(const py::list& arcs) {
  std::vector<rtdc_ckpt::Archive> out;
  for (auto item : arcs) {
    auto t = item.cast<py::tuple>();
    rtdc_ckpt::Archive a;
    a.raw = t[0].cast<bool>();
    a.recs = to_records(t[1].cast<py::list>());
    out.push_back(std::move(a));
  }
  return out;
}

// Per-step gradient bookkeeping of a flat parameter space, in one C++ pass instead of ~300
// Python property reads (`p.grad`, `data_ptr()`) between the end of backward and the
// optimizer launch: for each parameter, 0 = no gradient, 1 = gradient already is its slice of
// the flat buffer at `base + 4*offset`, 2 = gradient lives elsewhere (must be folded in).
static std::vector<int8_t> grad_status(const std::vector<at::Tensor>& params, int64_t base,
                                       const std::vector<int64_t>& offsets) {
  TORCH_CHECK(params.size() == offsets.size(), "grad_status: one offset per parameter");
  std::vector<int8_t> st(params.size(), 0);
  for (size_t i = 0; i < params.size(); ++i) {
    const at::Tensor& g = params[i].grad();
    if (!g.defined()) continue;
    st[i] = (reinterpret_cast<int64_t>(g.data_ptr()) == base + 4 * offsets[i]) ? 1 : 2;
  }
  return st;
}

// -> (file_size, [(archive_base, archive_size, [(abs_data_offset, size), ...]), ...])
static py::tuple plan_layout(const py::list& arcs) {
  auto a = to_archives(arcs);
  uint64_t total = rtdc_ckpt::layout_archives(a);
  py::list out;
  for (auto& x : a) {
    py::list recs;
    for (auto& r : x.recs) recs.append(py::make_tuple(x.base + r.data_off, rtdc_ckpt::rec_size(r)));
    out.append(py::make_tuple(x.base, x.size, recs));
  }
  return py::make_tuple(total, out);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  py::class_<rtdc_ddp::GradBucketEngine>(m, "GradBucketEngine")
      .def(py::init([](at::Tensor flat, std::vector<int64_t> bounds, std::vector<int64_t> param_bucket,
                       std::vector<std::pair<int64_t, int64_t>> seg, py::object pg, bool use_avg, double post_scale,
                       c10::optional<at::Tensor> comm_buf, int64_t zero_world, int64_t zero_rank) {
             auto cpg = pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>();
             return new rtdc_ddp::GradBucketEngine(flat, std::move(bounds), std::move(param_bucket), std::move(seg),
                                                   cpg, use_avg, post_scale, comm_buf, zero_world, zero_rank);
           }),
           py::arg("flat_grad"), py::arg("bounds"), py::arg("param_bucket"), py::arg("segments"),
           py::arg("process_group"), py::arg("use_avg"), py::arg("post_scale"), py::arg("comm_buf") = py::none(),
           py::arg("zero_world") = 0, py::arg("zero_rank") = 0)
      .def("comm_bytes_per_step", &rtdc_ddp::GradBucketEngine::comm_bytes_per_step)
      .def("mark_ready", &rtdc_ddp::GradBucketEngine::mark_ready)
      .def("finalize", &rtdc_ddp::GradBucketEngine::finalize, py::arg("defer_last") = false)
      .def("wait_tail", &rtdc_ddp::GradBucketEngine::wait_tail)
      .def("tail_pending", &rtdc_ddp::GradBucketEngine::tail_pending)
      .def("can_stream_wait", &rtdc_ddp::GradBucketEngine::can_stream_wait)
      .def("stream_wait_bucket", &rtdc_ddp::GradBucketEngine::stream_wait_bucket)
      .def("tail_start", &rtdc_ddp::GradBucketEngine::tail_start)
      .def("set_tail_split", &rtdc_ddp::GradBucketEngine::set_tail_split, py::arg("max_elems"))
      .def("tail_piece_starts", &rtdc_ddp::GradBucketEngine::tail_piece_starts)
      .def("wait_tail_piece", &rtdc_ddp::GradBucketEngine::wait_tail_piece, py::arg("i"))
      .def("num_buckets", &rtdc_ddp::GradBucketEngine::num_buckets)
      .def("launched", &rtdc_ddp::GradBucketEngine::launched)
      .def("steps", &rtdc_ddp::GradBucketEngine::steps)
      .def("bucket_bytes", &rtdc_ddp::GradBucketEngine::bucket_bytes)
      .def("set_p2p", &rtdc_ddp::GradBucketEngine::set_p2p, py::arg("comm"), py::arg("max_bytes"))
      .def("p2p_buckets", &rtdc_ddp::GradBucketEngine::p2p_buckets);
  py::class_<rtdc_p2p::P2PComm, std::shared_ptr<rtdc_p2p::P2PComm>>(m, "P2PComm")
      .def(py::init<int, int, long long, int, double, int>(), py::arg("rank"), py::arg("world"),
           py::arg("capacity_bytes"), py::arg("device"), py::arg("timeout_s") = 30.0, py::arg("blocks") = 32)
      .def("handle", &rtdc_p2p::P2PComm::handle)
      .def("open", &rtdc_p2p::P2PComm::open)
      .def("allreduce_", &rtdc_p2p::P2PComm::allreduce_, py::arg("tensor"), py::arg("average") = true)
      .def("error", &rtdc_p2p::P2PComm::error)
      .def("error_ptr", &rtdc_p2p::P2PComm::error_ptr)
      .def("snapshot_error", &rtdc_p2p::P2PComm::snapshot_error)
      .def("capacity", &rtdc_p2p::P2PComm::capacity)
      .def("epoch", &rtdc_p2p::P2PComm::epoch)
      .def_property_readonly("world", &rtdc_p2p::P2PComm::world)
      .def_property_readonly("rank", &rtdc_p2p::P2PComm::rank);

  m.doc() = "MI355X (gfx950) kernels and native checkpoint engine";
  m.def("gemm_bf16", &gemm_bf16);
  m.def("gemm_bf16_grouped", &gemm_bf16_grouped);
  m.def("gemm4b", &rtdc_gemm4b_set, py::arg("v") = -1,
        "route K-major x K-major 256x256 products to the one-barrier 4-wave kernel (1/0), or query (-1); returns the previous setting");
  m.def("gemm_f32", &gemm_f32);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("colsum_partial", &colsum_partial);
  m.def("colsum_multi", &colsum_multi);
  m.def("colsum", &colsum);
  m.def("xent", &xent);
  m.def("adamw", &adamw, py::arg("chunks"), py::arg("nchunks"), py::arg("p"), py::arg("g"), py::arg("m"),
        py::arg("v"), py::arg("shadow"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"),
        py::arg("bc1"), py::arg("bc2_sqrt"), py::arg("grad_scale"), py::arg("skip_ptr") = 0);
  m.def("sgd", &sgd, py::arg("chunks"), py::arg("nchunks"), py::arg("p"), py::arg("g"), py::arg("buf"),
        py::arg("shadow"), py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("wd"),
        py::arg("nesterov"), py::arg("first"), py::arg("grad_scale"), py::arg("skip_ptr") = 0);
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def("f32_to_bf16_t", &f32_to_bf16_t);
  m.def("bf16_transpose_multi", &bf16_transpose_multi);
  m.def("bf16_transpose_jobs_bytes", &rtdc_bf16_transpose_jobs_bytes);
  m.def("sumsq", &sumsq);
  m.def("softmax_fwd", &softmax_fwd);
  m.def("softmax_bwd", &softmax_bwd);
  m.def("embed_fwd", &embed_fwd);
  m.def("sort_ids", &sort_ids);
  m.def("synth_tokens", &synth_tokens);
  m.def("fill_f32", &fill_f32, py::arg("x"), py::arg("value") = 0.0);
  m.def("embed_bwd", &embed_bwd, py::arg("sidx"), py::arg("perm"), py::arg("dout"), py::arg("dwte"), py::arg("dwpe"),
        py::arg("B"), py::arg("T"), py::arg("accumulate_wpe"), py::arg("accumulate_wte") = false);
  m.def("dropout", &dropout);
  m.def("relu_dropout", &relu_dropout);
  m.def("flash_fwd", &flash_fwd);
  m.def("flash_bwd", &flash_bwd, py::arg("qkv"), py::arg("out"), py::arg("dout"), py::arg("lse"), py::arg("delta"),
        py::arg("dqkv"), py::arg("B"), py::arg("T"), py::arg("H"), py::arg("Hkv"), py::arg("Dh"), py::arg("scale"),
        py::arg("cs_ws") = py::none(), py::arg("part") = py::none(), py::arg("qs") = 1, py::arg("which") = 3,
        py::arg("delta_ready") = false);
  m.def("flash_delta", &flash_delta);
  m.def("rope", &rope);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("im2col", &im2col);
  m.def("conv_gemm", &conv_gemm);
  m.def("conv_gemm_bnb", &conv_gemm_bnb);
  m.def("col2im", &col2im);
  m.def("bn_fwd", &bn_fwd);
  m.def("bn_bwd", &bn_bwd);
  m.def("bn_relu_maxpool", &bn_relu_maxpool);
  m.def("stem_s2d", &stem_s2d);
  m.def("stem_w_s2d", &stem_w_s2d);
  m.def("stem_dw_s2d", &stem_dw_s2d);
  m.def("conv_w_flip_t", &conv_w_flip_t);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("xent_finalize", &xent_finalize);
  m.def("xent_alpha", &xent_alpha);
  m.def("scale_dev", &scale_dev);
  m.def("nchw_to_nhwc_bf16", &nchw_to_nhwc_bf16);
  m.def("copy2d", &copy2d);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("pool_bn_bwd", &pool_bn_bwd);
  m.def("avgpool", &avgpool);

  m.def("grad_status", &grad_status, "per-parameter gradient placement: 0 none, 1 flat slice, 2 elsewhere");
  m.def("have_gpu", &rtdc_ckpt::g_have_gpu);
  m.def("plan_layout", &plan_layout, "file layout of a list of (raw, records) archives");
  // the checkpoint writers' CRC-32 (PCLMUL folding, zlib-compatible; runtime/crc32_fast.h)
  m.def(
      "crc32",
      [](py::bytes b, uint32_t init) {
        std::string s = b;
        return rtdc::crc::crc32_fast(init, s.data(), s.size());
      },
      py::arg("data"), py::arg("init") = 0u);
  m.def(
      "read_ranges",
      [](const std::string& path, std::vector<uint64_t> offs, std::vector<uint64_t> lens, std::vector<uintptr_t> dsts,
         int nthreads) {
        py::gil_scoped_release nogil;
        rtdc_ckpt::read_ranges(path, offs, lens, dsts, nthreads);
      },
      "parallel pread of (offset, len) ranges into raw destination pointers");
  m.def(
      "zip_data_records",
      [](const std::string& path, std::vector<uint64_t> bases, std::vector<uint64_t> lens, int nthreads) {
        py::gil_scoped_release nogil;
        return rtdc_ckpt::zip_data_records(path, bases, lens, nthreads);
      },
      py::arg("path"), py::arg("bases"), py::arg("lengths"), py::arg("nthreads") = 8,
      "(data offset, size) of the '*/data/0' record of each zip archive slice [base, base + length)");

  py::class_<Engine>(m, "CkptEngine")
      .def(py::init<size_t, size_t, int, int, bool, uintptr_t>(), py::arg("nslots"), py::arg("slot_bytes"),
           py::arg("nwriters"), py::arg("device"), py::arg("direct_io") = true, py::arg("stream") = 0)
      .def(
          "submit",
          [](Engine& e, const py::list& files, uintptr_t ready_event) {
            std::vector<std::shared_ptr<FileJob>> fj;
            for (auto item : files) {
              auto t = item.cast<py::tuple>();
              auto f = std::make_shared<FileJob>();
              f->path = t[0].cast<std::string>();
              f->fsync_on = t[1].cast<bool>();
              f->crc_on = t[2].cast<bool>();
              f->archives = to_archives(t[3].cast<py::list>());
              fj.push_back(f);
            }
            return e.submit(std::move(fj), reinterpret_cast<hipEvent_t>(ready_event));
          },
          py::arg("files"), py::arg("ready_event") = 0)
      .def("poll", &Engine::poll)
      .def(
          "wait",
          [](Engine& e, int id) {
            py::gil_scoped_release nogil;
            return e.wait(id);
          })
      .def(
          "read_to_device",
          [](Engine& e, const std::string& path, std::vector<uint64_t> offs, std::vector<uint64_t> lens,
             std::vector<uintptr_t> dsts, int nthreads) {
            py::gil_scoped_release nogil;
            e.read_to_device(path, offs, lens, dsts, nthreads);
          },
          py::arg("path"), py::arg("offs"), py::arg("lens"), py::arg("dsts"), py::arg("nthreads") = 8)
      .def(
          "timings",
          [](Engine& e, int id) {
            py::gil_scoped_release nogil;
            return e.timings(id);
          },
          "(seconds to the last D2H piece in the pinned ring, seconds to durable) of a finished job")
      .def_property_readonly("d2h_mode", &Engine::d2h_mode)
      .def_property_readonly("slot_bytes", &Engine::slot_bytes)
      .def_property_readonly("pinned", &Engine::pinned);
}
