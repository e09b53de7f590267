// PyTorch bindings for the masters_thesis_amd HIP kernels (masters_thesis_amd._C).
// Kernels are plain HIP launchers (extern "C", raw pointers + hipStream_t); this file only
// validates tensors and forwards the current PyTorch HIP stream, so every op is stream-ordered
// with PyTorch and capturable into a HIP graph.
#include <torch/extension.h>

#include <cmath>
#include <map>
#include <tuple>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include "batch_gather.h"

extern "C" {
int mta_lstm_fwd_layer(int H, int prec, const float* x, const float* w_ih, const float* b_ih, const float* b_hh,
                       int fin, const float* gx, float* stash, const float* w_hh, float* hseq, int N, int Np, int T,
                       hipStream_t st);
int mta_lstm_bwd_layer(int H, int prec, const float* stash, const float* w_hh, const float* dH, const float* dh_last,
                       float* dG, int N, int Np, int T, hipStream_t st);
int mta_lstm_wgrad(int prec, const float* dG, const float* hseq, const float* inp, int inp_batch_first, int N, int Np,
                   int T, int H, int F, float* g_wih, float* g_whh, float* g_bih, float* g_bhh, float* part,
                   hipStream_t st);
long mta_lstm_wgrad_part_floats(int fused, int T, int H, int F);
int mta_gemm_f32(int prec, const float* A, const float* B, const float* bias, const float* mask, float* C, int M,
                 int N, int K, int b_kn, hipStream_t st);
int mta_gemm_f32x(int prec, const float* A, int a_km, int lda, const float* B, int b_kn, int ldb, float* C, int ldc,
                  int n_store, int M, int N, int K, int flags, const float* bias, float* pre, const float* mask, const float* resid, const uint64_t* seed, float drop_p, hipStream_t st);
void mta_colsum_f32(const float* A, int M, int N, int lda, float* out, hipStream_t st);
void mta_pair_colsum(const float* ab, int n, float* sa, float* sb, hipStream_t st);
int mta_attention_f32(int bwd, const float* qkv, const float* out, const float* dout, float* o, float* lse, float* dqkv,
                      int nseq, int T, int D, int heads, const float* rope, hipStream_t st);
void mta_seeds_advance(uint64_t* seeds, int n, hipStream_t st);
void mta_lstm_prep(const float* w_ih, const float* b_ih, const float* b_hh, int H, int F, float* w_um, float* b_um,
                   hipStream_t st);
void mta_gather_batch(const float* const* src, float* const* dst, const long* row_floats, int ntensors,
                      const int* perm, int* cursor, int* arrive, int B, int row_offset, hipStream_t st);
void mta_decoder_losses(const float* ab, const float* y, const float* factor, const float* inv_psi, int N, int n,
                        int C, int windows, int kwin, int factor_stride, int want_nll, float c_nll, float c_mse,
                        float batch_weight, float* out, float* gmse, float* gnll, double* acc, hipStream_t st);
int mta_heads_losses_train(const float* h, int H, const float* wa, const float* ba, const float* wb, const float* bb,
                           const float* y, const float* factor, const float* inv_psi, int N, int n, int C, int windows,
                           int kwin, int factor_stride, int want_nll, float c_nll, float c_mse, float batch_weight,
                           float* out, double* acc, float* dh, float* g_wa, float* g_ba, float* g_wb, float* g_bb,
                           int dh_rows, hipStream_t st);
void mta_heads_losses(const float* h, int H, const float* wa, const float* ba, const float* wb, const float* bb,
                      float* ab_out, const float* y, const float* factor, const float* inv_psi, int N, int n, int C,
                      int windows, int kwin, int factor_stride, int want_nll, float c_nll, float c_mse,
                      float batch_weight, float* out, float* gmse, float* gnll, double* acc, hipStream_t st);
void mta_heads_losses_bwd(const float* g_mse, const float* g_nll, const float* g_total, float c_nll, float c_mse, const float* gmse, const float* gnll,
                          int has_nll, const float* h, int N, int H, const float* wa, const float* wb, float* dh, float* dab,
                          float* g_wa, float* g_ba, float* g_wb, float* g_bb, float* part, hipStream_t st);
void mta_set_heads_deterministic(int on);
long mta_heads_part_floats(int N, int H);
int mta_optim_num_partials(long n);
void mta_grad_sqnorm(const float* g, long n, float scale, float* partials, float* step, hipStream_t st);
int mta_adam_fused_partials();
void mta_adam_fused(float* p, float* g, float* m, float* v, long n, float* partials, unsigned long long* ticket,
                    const float* lr, float* step, float beta1, float beta2, float eps, float wd, float max_norm,
                    float scale, int adamw, int zero_grad, float* norm_out, float* nonfinite, int n_cov,
                    const long* cov_s, const long* cov_e, const float* ext, int n_ext, int ext_only, hipStream_t st);
void mta_gemm_grad_producer(float* norm_parts, int overwrite);
int mta_gemm_norm_parts();
void mta_adam(float* p, float* g, float* m, float* v, long n, const float* partials, const float* lr,
              const float* step, float beta1, float beta2, float eps, float wd, float max_norm, float scale, int adamw,
              float* norm_out, float* nonfinite, hipStream_t st);
void mta_scale(float* x, long n, float s, hipStream_t st);
void mta_zero_bytes(void* dst, long bytes, hipStream_t st);
// gemm.hip / norm.hip / attention.hip (MLP + transformer encoders)
int mta_gemm_bf16(int mode, const void* A, const void* B, int M, int N, int K, int lda, int ldb, float alpha,
                  int flags, const float* bias, const float* resid, const void* aux_in, const uint64_t* seed,
                  float drop_p, void* out_bf16, float* out_f32, void* aux_pre, int ldc, int n_store, int ksplit,
                  float* bias_grad, int defer, hipStream_t st);
void mta_gemm_flush();
void mta_gemm_set_big(int on);
void mta_norm_flush();
void mta_norm_discard();
void mta_norm_defer();
void mta_gemm_group_flush();
void mta_gemm_group_discard();
int mta_cast_pad(int n, const float* const* src, void* const* dst, const int* rows, const int* cols,
                 const int* rows_p, const int* cols_p, const int* ld_src, uint64_t* seeds, int nseeds, hipStream_t st);
int mta_norm(int bwd, const void* x, int x_bf16, int ldx, int M, int D, int rms, float eps, const float* gamma,
             const float* beta, void* y_bf16, float* y_f32, float* mean, float* rstd, const uint64_t* seed,
             float drop_p, const void* dy, int dy_bf16, const float* dres, const void* pre, int pre_f32, void* dx_bf16,
             float* dx_f32, float* dgamma, float* dbeta, const float* hw_a, const float* hb_a, const float* hw_b, const float* hb_b,
             float* ab, int ab_rows, float* g_wa, float* g_wb, hipStream_t st);
int mta_tr_ffn(int backward, int M, int d, int dff, float eps, const void* w1, const void* w2, const float* b1,
               const float* b2, const float* g2, const float* x1, const uint64_t* seed, float drop_p, void* xn2,
               void* pre, void* u, float* r2, float* x2, const void* dxb, const float* dx, const float* r2in,
               const void* prein, void* dpre, float* dx1, void* dx1b, float* dg2, void* uT, void* xn2T, void* dpreT,
               void* dxT, hipStream_t st);
int mta_frag_pack(int count, const float* const* src, void* const* dst, const int* n, const int* k, const int* tr,
                  int ncast, const float* const* csrc, void* const* cdst, const int* crows, const int* ccols,
                  const int* crows_p, const int* ccols_p, const int* cld, uint64_t* seeds, int nseeds,
                  hipStream_t st);
int mta_tr_attn_dx(int M, const void* dqkv, const void* wqkvt, const float* x, const float* r1, const float* g1,
                   const float* dx1, float* dx, void* dxb, float* dg1, hipStream_t st);
int mta_tr_attn_fwd(int nseq, int T, int d, int heads, const float* x, const void* wqkv, const void* wo, const float* g1,
                    const float* bqkv, const float* bo, const float* rope, float eps, void* xn, float* r1, void* qkv,
                    void* o, float* lse, float* x1, const float* in, const float* we, const float* be, int F, int rows_in,
                    float* x_out, hipStream_t st);
int mta_tr_transpose_bf16(int n, const void* const* src, void* const* dst, const int* rows, const int* cols,
                          hipStream_t st);
int mta_attention(int bwd, const void* qkv, void* out, float* lse, const void* dout, void* dqkv, int nseq, int T,
                  int D, int heads, float rope_base, const float* rope, const void* dx1, const void* wot, hipStream_t st);
// lstm_stack.hip (layer-pipelined multi-layer LSTM)
int mta_lstm_stack_fwd_g(int H, int prec, int L, int fin, const float* x, const float* const* w_ih,
                         const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                         float* const* hseq, float* const* xdrop, uint32_t* const* mask, float* const* stash,
                         const uint64_t* seeds, float drop_p, unsigned* flags, int N, int Np, int T,
                         const MtaBatchGather* gather, unsigned long long* gran, int decoupled, hipStream_t st);
int mta_lstm_stack_fwd(int H, int prec, int L, int fin, const float* x, const float* const* w_ih,
                       const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                       float* const* hseq, float* const* xdrop, uint32_t* const* mask, float* const* stash,
                       const uint64_t* seeds, float drop_p, unsigned* flags, int N, int Np, int T,
                       unsigned long long* gran, int decoupled, hipStream_t st);
int mta_lstm_stack_bwd(int H, int prec, int L, int fin, const float* const* stash, const float* const* w_hh,
                       const float* const* w_ih, const float* dh_last, float* const* dG, float* const* dX,
                       const float* const* hseq, const float* const* inp, float* const* g_wih, float* const* g_whh,
                       float* const* g_bih, float* const* g_bhh, const uint32_t* const* mask, float* const* part,
                       uint64_t* seeds, float drop_p, int dropout, unsigned* flags, int N, int Np, int T,
                       int form, hipStream_t st);
long mta_lstm_stack_flag_words(int Np);
int mta_lstm_stack_epoch_shift(int T);
// allreduce.hip (one-shot / two-shot all-reduce over xGMI peer memory, one channel per bucket)
int mta_xgmi_alloc(long bytes, void** out);
int mta_xgmi_free(void* p);
int mta_xgmi_ipc_handle(void* p, unsigned char* out64);
int mta_xgmi_ipc_open(const unsigned char* in64, void** out);
int mta_xgmi_ipc_close(void* p);
long mta_xgmi_buffer_bytes(int world, long cap, int channels);
int mta_xgmi_ctl_words();
int mta_xgmi_max_channels();
int mta_xgmi_timeout_word();
int mta_xgmi_allreduce(float* grad, long n, long off, long cap, int channel, int channels, int twoshot,
                       void* const* bufs, int rank, int world, unsigned* ctl, float* sq, hipStream_t st);
int mta_xgmi_max_blocks();
// data.hip (dataset build)
int mta_dgp(uint64_t seed, int n_stocks, long n_samples, int mkt_df, float mkt_loc, float mkt_scale, int idio_df,
            float idio_loc, float idio_scale, float a_loc, float a_scale, float b_loc, float b_scale, float* r_market,
            float* r_stocks, float* alphas, float* betas, hipStream_t st);
void mta_ols_features(const float* target, int W, int K, int n, int C, float* alphas, float* betas, float* factor,
                      float* inv_psi, hipStream_t st);
// host/prefetch.cpp
void* mta_prefetch_create(int ntensors, const void* const* host, const long* row_bytes, void* const* staging, int B,
                          int R, int nthreads);
void mta_prefetch_start(void* h, const long* idx, long n_idx, long n_batches);
int mta_prefetch_wait(void* h, long batch, long timeout_ms);
int mta_prefetch_ready(void* h, long batch);
void mta_prefetch_release(void* h, long batch);
void mta_prefetch_stop(void* h);
void mta_prefetch_destroy(void* h);
}

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

// one statement (do / while): an unbraced `if (x) CHECK_F32(*x);` must not run the later checks on an empty x
#define CHECK_F32(t)                                                                            \
  do {                                                                                              \
    TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor");                                         \
    TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32");                            \
    TORCH_CHECK((t).is_contiguous(), #t " must be contiguous");                                     \
  } while (0)

using OptT = c10::optional<at::Tensor>;

bool has(const OptT& t) { return t.has_value() && t->defined(); }

const float* opt_ptr(const OptT& t) {
  if (!has(t)) return nullptr;
  CHECK_F32(*t);
  return t->data_ptr<float>();
}

float* opt_mut(const OptT& t) { return const_cast<float*>(opt_ptr(t)); }

// ------------------------------------------------------------------------------------------- LSTM
void lstm_fwd_layer(int64_t H, int64_t prec, const OptT& x, const OptT& w_ih, const OptT& b_ih, const OptT& b_hh,
                    const OptT& gx, const OptT& stash, at::Tensor w_hh, at::Tensor hseq, int64_t N, int64_t Np,
                    int64_t T) {
  CHECK_F32(w_hh);
  CHECK_F32(hseq);
  TORCH_CHECK(Np % 16 == 0 && N <= Np && N >= 1, "Np must be a multiple of 16 and >= N");
  TORCH_CHECK(hseq.numel() == T * Np * H, "hseq must be (T, Np, H)");
  TORCH_CHECK(w_hh.numel() == 4 * H * H, "w_hh must be (4H, H)");
  if (has(stash)) TORCH_CHECK(stash->numel() == T * Np * 5 * H, "stash must hold T*Np*5H floats");
  int fin = 0;
  if (has(x)) {
    TORCH_CHECK(x->dim() == 3 && x->size(0) == N && x->size(1) == T, "x must be (N, T, F)");
    fin = (int)x->size(2);
    TORCH_CHECK(fin == 3 || fin == 5, "fused input projection supports F in {3, 5}");
    TORCH_CHECK(has(w_ih) && w_ih->numel() == 4 * H * fin, "w_ih must be (4H, F)");
    TORCH_CHECK(has(b_ih) && has(b_hh), "fused input projection needs b_ih and b_hh");
  } else {
    TORCH_CHECK(has(gx) && gx->numel() == T * Np * 4 * H, "gx must be (T, Np, 4H)");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(hseq.device());
  int rc = mta_lstm_fwd_layer((int)H, (int)prec, opt_ptr(x), opt_ptr(w_ih), opt_ptr(b_ih), opt_ptr(b_hh), fin,
                              opt_ptr(gx), opt_mut(stash), w_hh.data_ptr<float>(), hseq.data_ptr<float>(), (int)N,
                              (int)Np, (int)T, cur_stream());
  TORCH_CHECK(rc == 0, "lstm_fwd_layer: unsupported configuration (H must be 32, 64 or 128)");
}

void lstm_bwd_layer(int64_t H, int64_t prec, at::Tensor stash, at::Tensor w_hh, const OptT& dH, const OptT& dh_last,
                    at::Tensor dG, int64_t N, int64_t Np, int64_t T) {
  CHECK_F32(stash);
  CHECK_F32(w_hh);
  CHECK_F32(dG);
  TORCH_CHECK(stash.numel() == T * Np * 5 * H && dG.numel() == T * Np * 4 * H, "bad stash/dG shape");
  const bool has_dh = has(dH);
  if (has_dh) {
    TORCH_CHECK(dH->numel() == T * Np * H, "dH must be (T, Np, H)");
  } else {
    TORCH_CHECK(has(dh_last) && dh_last->numel() == N * H, "dh_last must be (N, H)");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dG.device());
  int rc = mta_lstm_bwd_layer((int)H, (int)prec, stash.data_ptr<float>(), w_hh.data_ptr<float>(), opt_ptr(dH),
                              has_dh ? nullptr : opt_ptr(dh_last), dG.data_ptr<float>(), (int)N, (int)Np, (int)T,
                              cur_stream());
  TORCH_CHECK(rc == 0, "lstm_bwd_layer: unsupported configuration");
}

void lstm_wgrad(int64_t prec, at::Tensor dG, at::Tensor hseq, at::Tensor inp, bool inp_batch_first, int64_t N, int64_t Np,
                int64_t T, int64_t H, at::Tensor g_wih, at::Tensor g_whh, at::Tensor g_bih, at::Tensor g_bhh,
                const OptT& part) {
  CHECK_F32(dG);
  CHECK_F32(hseq);
  CHECK_F32(inp);
  CHECK_F32(g_wih);
  CHECK_F32(g_whh);
  CHECK_F32(g_bih);
  CHECK_F32(g_bhh);
  const int64_t F = g_wih.numel() / (4 * H);
  TORCH_CHECK(dG.numel() == T * Np * 4 * H && hseq.numel() == T * Np * H, "bad dG/hseq shape");
  TORCH_CHECK(inp.numel() == (inp_batch_first ? N * T * F : T * Np * F), "bad layer-input shape");
  TORCH_CHECK(g_whh.numel() == 4 * H * H && g_bih.numel() == 4 * H && g_bhh.numel() == 4 * H, "bad grad shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dG.device());
  const int rc = mta_lstm_wgrad((int)prec, dG.data_ptr<float>(), hseq.data_ptr<float>(), inp.data_ptr<float>(),
                                inp_batch_first ? 1 : 0, (int)N, (int)Np, (int)T, (int)H, (int)F,
                                g_wih.data_ptr<float>(), g_whh.data_ptr<float>(), g_bih.data_ptr<float>(),
                                g_bhh.data_ptr<float>(), opt_mut(part), cur_stream());
  TORCH_CHECK(rc == 0, "lstm_wgrad: unsupported configuration (H=", H, ", F=", F, ")");
}

// 32-true extras GEMM (csrc/gemm_f32.hip mta_gemm_f32x): C[:M, :n_store] (=|+=) op(A) . op(B)^T (+ bias, GELU with
// its input saved to pre); A viewed [M][K] (lda) or stored [K][M] (a_km); B [N][K] or [K][N] (b_kn)
void gemm_f32x(int64_t prec, at::Tensor A, bool a_km, int64_t lda, at::Tensor B, bool b_kn, int64_t ldb, at::Tensor C,
               int64_t ldc, int64_t n_store, int64_t M, int64_t N, int64_t K, int64_t flags,
               c10::optional<at::Tensor> bias, c10::optional<at::Tensor> pre, c10::optional<at::Tensor> mask,
               c10::optional<at::Tensor> resid, c10::optional<at::Tensor> seed, double drop_p) {
  for (at::Tensor* t : {&A, &B, &C}) TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat, "gemm_f32x: fp32 GPU");
  TORCH_CHECK(A.numel() >= (a_km ? (K - 1) * lda + M : (M - 1) * lda + K), "gemm_f32x: A too small");
  TORCH_CHECK(B.numel() >= (b_kn ? (K - 1) * ldb + N : (N - 1) * ldb + K), "gemm_f32x: B too small");
  TORCH_CHECK(C.numel() >= (M - 1) * ldc + n_store, "gemm_f32x: C too small");
  if (bias.has_value()) TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->numel() >= N, "bias");
  if (pre.has_value()) TORCH_CHECK(pre->is_cuda() && pre->scalar_type() == at::kFloat && pre->numel() >= (M - 1) * ldc + n_store, "pre");
  if (mask.has_value()) TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kFloat && mask->numel() >= M * N, "mask");
  if (resid.has_value())
    TORCH_CHECK(resid->is_cuda() && resid->scalar_type() == at::kFloat && resid->numel() >= (M - 1) * ldc + n_store, "resid");
  if (seed.has_value()) TORCH_CHECK(seed->is_cuda() && seed->scalar_type() == at::kLong && seed->numel() >= 1, "seed");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const int rc = mta_gemm_f32x((int)prec, A.data_ptr<float>(), a_km ? 1 : 0, (int)lda, B.data_ptr<float>(), b_kn ? 1 : 0,
                               (int)ldb, C.data_ptr<float>(), (int)ldc, (int)n_store, (int)M, (int)N, (int)K, (int)flags,
                               bias.has_value() ? bias->data_ptr<float>() : nullptr,
                               pre.has_value() ? pre->data_ptr<float>() : nullptr,
                               mask.has_value() ? mask->data_ptr<float>() : nullptr,
                               resid.has_value() ? resid->data_ptr<float>() : nullptr,
                               seed.has_value() ? reinterpret_cast<const uint64_t*>(seed->data_ptr<int64_t>()) : nullptr,
                               (float)drop_p, cur_stream());
  TORCH_CHECK(rc == 0, "gemm_f32x: unsupported configuration (", rc, ")");
}

// out[:N] += column sums of A[:M][:N] (lda): bias gradients of the 32-true extras
// sa += sum of ab[:, 0], sb += sum of ab[:, 1] (ab: contiguous (n, 2) fp32)
void pair_colsum(at::Tensor ab, int64_t n, at::Tensor sa, at::Tensor sb) {
  TORCH_CHECK(ab.is_cuda() && ab.scalar_type() == at::kFloat && ab.is_contiguous() && ab.numel() >= 2 * n,
              "pair_colsum: contiguous (n, 2) fp32 GPU tensor");
  CHECK_F32(sa);
  CHECK_F32(sb);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(ab.device());
  mta_pair_colsum(ab.data_ptr<float>(), (int)n, sa.data_ptr<float>(), sb.data_ptr<float>(), cur_stream());
}

void colsum_f32(at::Tensor A, int64_t M, int64_t N, int64_t lda, at::Tensor out) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == at::kFloat && out.is_cuda() && out.scalar_type() == at::kFloat &&
              out.numel() >= N && A.numel() >= (M - 1) * lda + N, "colsum_f32: fp32 GPU tensors");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  mta_colsum_f32(A.data_ptr<float>(), (int)M, (int)N, (int)lda, out.data_ptr<float>(), cur_stream());
}

// C = A . B^T (+ bias) (* mask); B is [N][K], or [K][N] with b_kn (csrc/gemm_f32.hip)
void gemm_f32(int64_t prec, at::Tensor A, at::Tensor B, at::Tensor C, c10::optional<at::Tensor> bias,
              c10::optional<at::Tensor> mask, bool b_kn) {
  CHECK_F32(A);
  CHECK_F32(B);
  CHECK_F32(C);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_f32: 2-D operands");
  const int64_t M = A.size(0), K = A.size(1), N = b_kn ? B.size(1) : B.size(0);
  TORCH_CHECK((b_kn ? B.size(0) : B.size(1)) == K && C.size(0) == M && C.size(1) == N, "gemm_f32: shape mismatch");
  const float* pb = nullptr;
  const float* pm = nullptr;
  if (bias && bias->defined()) {
    CHECK_F32((*bias));
    TORCH_CHECK(bias->numel() == N, "gemm_f32: bias[N]");
    pb = bias->data_ptr<float>();
  }
  if (mask && mask->defined()) {
    CHECK_F32((*mask));
    TORCH_CHECK(mask->numel() == M * N, "gemm_f32: mask[M][N]");
    pm = mask->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const int rc = mta_gemm_f32((int)prec, A.data_ptr<float>(), B.data_ptr<float>(), pb, pm, C.data_ptr<float>(),
                              (int)M, (int)N, (int)K, b_kn ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "gemm_f32: unsupported configuration (", rc, ")");
}

void lstm_prep(at::Tensor w_ih, at::Tensor b_ih, at::Tensor b_hh, int64_t H, at::Tensor w_um, at::Tensor b_um) {
  CHECK_F32(w_ih);
  CHECK_F32(b_ih);
  CHECK_F32(b_hh);
  CHECK_F32(w_um);
  CHECK_F32(b_um);
  const int64_t F = w_ih.numel() / (4 * H);
  TORCH_CHECK(w_um.numel() == w_ih.numel() && b_um.numel() == 4 * H, "bad prep shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w_ih.device());
  mta_lstm_prep(w_ih.data_ptr<float>(), b_ih.data_ptr<float>(), b_hh.data_ptr<float>(), (int)H, (int)F,
                w_um.data_ptr<float>(), b_um.data_ptr<float>(), cur_stream());
}

// ------------------------------------------------------------------------------------------- data
void gather_batch(std::vector<at::Tensor> src, std::vector<at::Tensor> dst, at::Tensor perm, at::Tensor cursor,
                  at::Tensor arrive, int64_t B, int64_t row_offset) {
  TORCH_CHECK(src.size() == dst.size() && src.size() >= 1 && src.size() <= 4, "1..4 tensors");
  TORCH_CHECK(perm.scalar_type() == at::kInt && cursor.scalar_type() == at::kInt && arrive.scalar_type() == at::kInt,
              "perm/cursor/arrive must be int32");
  TORCH_CHECK(arrive.is_cuda() && arrive.numel() >= 65 * 32, "arrive: 65 x 32 int32 words (top + 64 sub-counters, one line each)");
  const float* s[4];
  float* d[4];
  long rf[4];
  for (size_t k = 0; k < src.size(); ++k) {
    CHECK_F32(src[k]);
    CHECK_F32(dst[k]);
    rf[k] = (long)(src[k].numel() / src[k].size(0));
    TORCH_CHECK(dst[k].numel() == B * rf[k], "dst ", k, " must hold B rows");
    s[k] = src[k].data_ptr<float>();
    d[k] = dst[k].data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(perm.device());
  mta_gather_batch(s, d, rf, (int)src.size(), perm.data_ptr<int>(), cursor.data_ptr<int>(), arrive.data_ptr<int>(),
                   (int)B, (int)row_offset, cur_stream());
}

// ------------------------------------------------------------------------------------------- losses
double* opt_acc(const OptT& acc) {
  if (!has(acc)) return nullptr;
  TORCH_CHECK(acc->is_cuda() && acc->scalar_type() == at::kDouble && acc->is_contiguous() && acc->numel() >= 8,
              "acc must be a contiguous float64 GPU tensor of >= 8 elements");
  return acc->data_ptr<double>();
}

void check_loss_inputs(int64_t N, const at::Tensor& y, const at::Tensor& factor, const at::Tensor& inv_psi,
                       int64_t windows, int64_t kwin, int64_t factor_stride, const at::Tensor& out,
                       const at::Tensor& gmse, const at::Tensor& gnll) {
  CHECK_F32(y);
  CHECK_F32(factor);
  CHECK_F32(inv_psi);
  CHECK_F32(out);
  CHECK_F32(gmse);
  CHECK_F32(gnll);
  TORCH_CHECK(y.dim() == 3 && y.size(0) == N && y.size(2) >= 2, "y must be (N, n, C>=2)");
  TORCH_CHECK(inv_psi.numel() == N, "inv_psi must be (N,)");
  TORCH_CHECK(windows * kwin == N, "windows * kwin must equal N");
  TORCH_CHECK(factor.numel() >= 2 + (windows - 1) * factor_stride, "factor too small");
  TORCH_CHECK(out.numel() >= 4 && gmse.numel() == 2 * N && gnll.numel() == 2 * N, "bad output shapes");
}

void decoder_losses(at::Tensor ab, at::Tensor y, at::Tensor factor, at::Tensor inv_psi, int64_t windows, int64_t kwin,
                    int64_t factor_stride, bool want_nll, double c_nll, double c_mse, double batch_weight,
                    at::Tensor out, at::Tensor gmse, at::Tensor gnll, const OptT& acc) {
  CHECK_F32(ab);
  const int64_t N = ab.size(0);
  TORCH_CHECK(ab.dim() == 2 && ab.size(1) == 2, "ab must be (N, 2)");
  check_loss_inputs(N, y, factor, inv_psi, windows, kwin, factor_stride, out, gmse, gnll);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(ab.device());
  mta_decoder_losses(ab.data_ptr<float>(), y.data_ptr<float>(), factor.data_ptr<float>(), inv_psi.data_ptr<float>(),
                     (int)N, (int)y.size(1), (int)y.size(2), (int)windows, (int)kwin, (int)factor_stride,
                     want_nll ? 1 : 0, (float)c_nll, (float)c_mse, (float)batch_weight, out.data_ptr<float>(),
                     gmse.data_ptr<float>(), gnll.data_ptr<float>(), opt_acc(acc), cur_stream());
}

void heads_losses(at::Tensor h, at::Tensor wa, at::Tensor ba, at::Tensor wb, at::Tensor bb, at::Tensor ab_out,
                  at::Tensor y, at::Tensor factor, at::Tensor inv_psi, int64_t windows, int64_t kwin,
                  int64_t factor_stride, bool want_nll, double c_nll, double c_mse, double batch_weight,
                  at::Tensor out, at::Tensor gmse, at::Tensor gnll, const OptT& acc) {
  CHECK_F32(h);
  CHECK_F32(wa);
  CHECK_F32(ba);
  CHECK_F32(wb);
  CHECK_F32(bb);
  CHECK_F32(ab_out);
  TORCH_CHECK(h.dim() == 2, "h must be (N, H)");
  const int64_t N = h.size(0), H = h.size(1);
  TORCH_CHECK(wa.numel() == H && wb.numel() == H && ba.numel() == 1 && bb.numel() == 1, "bad head shapes");
  TORCH_CHECK(ab_out.numel() == 2 * N, "ab_out must be (N, 2)");
  check_loss_inputs(N, y, factor, inv_psi, windows, kwin, factor_stride, out, gmse, gnll);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  mta_heads_losses(h.data_ptr<float>(), (int)H, wa.data_ptr<float>(), ba.data_ptr<float>(), wb.data_ptr<float>(),
                   bb.data_ptr<float>(), ab_out.data_ptr<float>(), y.data_ptr<float>(), factor.data_ptr<float>(),
                   inv_psi.data_ptr<float>(), (int)N, (int)y.size(1), (int)y.size(2), (int)windows, (int)kwin,
                   (int)factor_stride, want_nll ? 1 : 0, (float)c_nll, (float)c_mse, (float)batch_weight,
                   out.data_ptr<float>(), gmse.data_ptr<float>(), gnll.data_ptr<float>(), opt_acc(acc),
                   cur_stream());
}

// the training step's decoder in one launch (upstream gradient 1 on the total loss): losses + metrics into
// out / acc, dh (N, H) for the encoder, head gradients accumulated into g_*; false = too large (use the pair)
bool heads_losses_train(at::Tensor h, at::Tensor wa, at::Tensor ba, at::Tensor wb, at::Tensor bb, at::Tensor y,
                        at::Tensor factor, at::Tensor inv_psi, int64_t windows, int64_t kwin, int64_t factor_stride,
                        bool want_nll, double c_nll, double c_mse, double batch_weight, at::Tensor out,
                        const OptT& acc, at::Tensor dh, at::Tensor g_wa, at::Tensor g_ba, at::Tensor g_wb,
                        at::Tensor g_bb) {
  CHECK_F32(h);
  CHECK_F32(dh);
  CHECK_F32(g_wa);
  CHECK_F32(g_ba);
  CHECK_F32(g_wb);
  CHECK_F32(g_bb);
  TORCH_CHECK(h.dim() == 2, "h must be (N, H)");
  const int64_t N = h.size(0), H = h.size(1);
  TORCH_CHECK(wa.numel() == H && wb.numel() == H && ba.numel() == 1 && bb.numel() == 1, "bad head shapes");
  // dh may hold padded rows beyond N (the MLP encoder's 16-row padding): the launch zero-fills them
  TORCH_CHECK(dh.numel() >= N * H && dh.numel() % H == 0 && g_wa.numel() == H && g_wb.numel() == H && g_ba.numel() == 1 &&
                  g_bb.numel() == 1, "dh / head gradient shapes");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kFloat && y.is_contiguous() && y.dim() == 3 && y.size(0) == N &&
                  y.size(2) >= 2, "y must be (N, n, C >= 2) fp32");
  TORCH_CHECK(out.is_cuda() && out.numel() >= 4, "out: float[4]");
  TORCH_CHECK(windows * kwin == N, "windows * kwin must equal N");
  CHECK_F32(factor);
  CHECK_F32(inv_psi);
  TORCH_CHECK(inv_psi.numel() == N, "inv_psi must be (N,)");
  TORCH_CHECK(factor.numel() >= 2 + (windows - 1) * factor_stride, "factor too small");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  const int rc = mta_heads_losses_train(
      h.data_ptr<float>(), (int)H, wa.data_ptr<float>(), ba.data_ptr<float>(), wb.data_ptr<float>(),
      bb.data_ptr<float>(), y.data_ptr<float>(), factor.data_ptr<float>(), inv_psi.data_ptr<float>(), (int)N,
      (int)y.size(1), (int)y.size(2), (int)windows, (int)kwin, (int)factor_stride, want_nll ? 1 : 0, (float)c_nll,
      (float)c_mse, (float)batch_weight, out.data_ptr<float>(), opt_acc(acc), dh.data_ptr<float>(),
      g_wa.data_ptr<float>(), g_ba.data_ptr<float>(), g_wb.data_ptr<float>(), g_bb.data_ptr<float>(),
      (int)(dh.numel() / H), cur_stream());
  return rc == 0;
}

void heads_losses_bwd(const OptT& g_mse, const OptT& g_nll, const OptT& g_total, double c_nll, double c_mse,
                      at::Tensor gmse, at::Tensor gnll, bool has_nll, const OptT& h, const OptT& wa, const OptT& wb, const OptT& dh, const OptT& dab,
                      const OptT& g_wa, const OptT& g_ba, const OptT& g_wb, const OptT& g_bb) {
  CHECK_F32(gmse);
  CHECK_F32(gnll);
  const int64_t N = gmse.numel() / 2;
  int64_t H = 0;
  if (has(h)) {
    H = h->size(1);
    TORCH_CHECK(h->size(0) == N && has(wa) && has(wb), "heads backward needs h, wa, wb");
    if (has(dh)) TORCH_CHECK(dh->numel() == N * H, "dh must be (N, H)");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gmse.device());
  // the grid-parallel path of wide heads stages d(alpha, beta) in global memory
  at::Tensor dab_buf = has(dab) ? *dab : at::empty({2 * N}, gmse.options());
  // deterministic mode: per-block partials of the head parameter gradients, summed in block order
  const long np = mta_heads_part_floats((int)N, (int)H);
  at::Tensor part = np > 0 ? at::empty({np}, gmse.options()) : at::Tensor();
  mta_heads_losses_bwd(opt_ptr(g_mse), opt_ptr(g_nll), opt_ptr(g_total), (float)c_nll, (float)c_mse, gmse.data_ptr<float>(),
                       gnll.data_ptr<float>(), has_nll ? 1 : 0, opt_ptr(h), (int)N, (int)H, opt_ptr(wa), opt_ptr(wb),
                       opt_mut(dh), dab_buf.data_ptr<float>(), opt_mut(g_wa), opt_mut(g_ba), opt_mut(g_wb),
                       opt_mut(g_bb), np > 0 ? part.data_ptr<float>() : nullptr, cur_stream());
}

// ------------------------------------------------------------------------------------------- optimizer
int64_t optim_num_partials(int64_t n) { return mta_optim_num_partials((long)n); }

void grad_sqnorm(at::Tensor g, double scale, at::Tensor partials, const OptT& step) {
  CHECK_F32(g);
  CHECK_F32(partials);
  TORCH_CHECK(g.numel() % 4 == 0, "flat buffers must be padded to a multiple of 4");
  TORCH_CHECK(partials.numel() >= mta_optim_num_partials((long)g.numel()), "partials too small");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  mta_grad_sqnorm(g.data_ptr<float>(), (long)g.numel(), (float)scale, partials.data_ptr<float>(), opt_mut(step),
                  cur_stream());
}

void adam(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor partials, at::Tensor lr, at::Tensor step,
          double beta1, double beta2, double eps, double wd, double max_norm, double scale, bool adamw,
          const OptT& norm_out, const OptT& nonfinite) {
  CHECK_F32(p);
  CHECK_F32(g);
  CHECK_F32(m);
  CHECK_F32(v);
  CHECK_F32(partials);
  CHECK_F32(lr);
  CHECK_F32(step);
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && n % 4 == 0, "flat buffer size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  mta_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), (long)n,
           partials.data_ptr<float>(), lr.data_ptr<float>(), step.data_ptr<float>(), (float)beta1, (float)beta2,
           (float)eps, (float)wd, (float)max_norm, (float)scale, adamw ? 1 : 0, opt_mut(norm_out), opt_mut(nonfinite),
           cur_stream());
}

int64_t adam_fused_partials() { return mta_adam_fused_partials(); }

// one launch: grad norm + clip + Adam/AdamW (+ grad zeroing); ticket is an int64[1] zero-initialised once
void adam_fused(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor partials, at::Tensor ticket,
                at::Tensor lr, at::Tensor step, double beta1, double beta2, double eps, double wd, double max_norm,
                double scale, bool adamw, bool zero_grad, const OptT& norm_out, const OptT& nonfinite,
                std::vector<int64_t> cov_s, std::vector<int64_t> cov_e, const OptT& ext, bool ext_only) {
  CHECK_F32(p);
  CHECK_F32(g);
  CHECK_F32(m);
  CHECK_F32(v);
  CHECK_F32(partials);
  CHECK_F32(lr);
  CHECK_F32(step);
  TORCH_CHECK(ticket.is_cuda() && ticket.scalar_type() == at::kLong && ticket.numel() >= 1, "ticket: int64[1]");
  TORCH_CHECK(partials.numel() >= mta_adam_fused_partials(), "partials too small");
  TORCH_CHECK(!has(nonfinite) || nonfinite->numel() >= 2, "nonfinite needs 2 floats");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && n % 4 == 0, "flat buffer size mismatch");
  TORCH_CHECK(cov_s.size() == cov_e.size() && cov_s.size() <= 8, "adam_fused: at most 8 covered ranges");
  for (size_t k = 0; k < cov_s.size(); ++k)
    TORCH_CHECK(0 <= cov_s[k] && cov_s[k] <= cov_e[k] && cov_e[k] <= n / 4, "adam_fused: covered range out of bounds");
  TORCH_CHECK(cov_s.empty() || has(ext), "adam_fused: covered ranges need their producer partials");
  // ext_only: ext holds the squares of the WHOLE gradient (the xGMI all-reduce's partials): no norm pass at all;
  // the covered ranges then only mark what is left unzeroed
  TORCH_CHECK(!ext_only || has(ext), "adam_fused: ext_only needs ext");
  if (has(ext)) {
    CHECK_F32(*ext);
  }
  std::vector<long> cs(cov_s.begin(), cov_s.end()), ce(cov_e.begin(), cov_e.end());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  mta_adam_fused(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), (long)n,
                 partials.data_ptr<float>(), reinterpret_cast<unsigned long long*>(ticket.data_ptr<int64_t>()),
                 lr.data_ptr<float>(), step.data_ptr<float>(), (float)beta1, (float)beta2, (float)eps, (float)wd,
                 (float)max_norm, (float)scale, adamw ? 1 : 0, zero_grad ? 1 : 0, opt_mut(norm_out),
                 opt_mut(nonfinite), (int)cs.size(), cs.data(), ce.data(),
                 has(ext) ? ext->data_ptr<float>() : nullptr,
                 // every partial the caller passes is summed (FusedAdam.step hands over slots [0, last used slot],
                 // the unowned ones zeroed)
                 has(ext) ? (int)ext->numel() : 0, ext_only ? 1 : 0,
                 cur_stream());
}

// the next weight-gradient GEMM overwrites its output (no += onto a range the optimizer did not zero) and writes the
// clip-norm partials of it into parts[0 .. gemm_norm_parts())
void gemm_grad_producer(const OptT& parts, bool overwrite) {
  if (has(parts)) {
    CHECK_F32(*parts);
    TORCH_CHECK(parts->numel() >= mta_gemm_norm_parts(), "gemm_grad_producer: parts too small");
  }
  mta_gemm_grad_producer(has(parts) ? parts->data_ptr<float>() : nullptr, overwrite ? 1 : 0);
}

void scale_(at::Tensor x, double s) {
  CHECK_F32(x);
  TORCH_CHECK(x.numel() % 4 == 0, "flat buffers must be padded to a multiple of 4");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  mta_scale(x.data_ptr<float>(), (long)x.numel(), (float)s, cur_stream());
}

}  // namespace


// ------------------------------------------------------------------------------- MLP / transformer extras
#define CHECK_GPU(t, dt)                                                                        \
  do {                                                                                              \
    TORCH_CHECK((t).is_cuda() && (t).scalar_type() == (dt), #t " must be a GPU tensor of " #dt);   \
    TORCH_CHECK((t).is_contiguous(), #t " must be contiguous");                                     \
  } while (0)

template <class T>
T* opt_typed(const OptT& t, at::ScalarType dt, const char* name) {
  if (!has(t)) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == dt && t->is_contiguous(), name, ": bad tensor (device/dtype/layout)");
  return static_cast<T*>(t->data_ptr());
}

void check_span(const at::Tensor& t, int64_t rows, int64_t ld, int64_t cols, const char* name) {
  TORCH_CHECK(rows == 0 || t.numel() >= (rows - 1) * ld + cols, name, ": tensor too small for [", rows, "][", ld,
              "] access of ", cols, " columns");
}

void gemm_bf16(int64_t mode, at::Tensor A, at::Tensor B, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
               double alpha, int64_t flags, const OptT& bias, const OptT& resid, const OptT& aux_in, const OptT& seed,
               double drop_p, const OptT& out_bf16, const OptT& out_f32, const OptT& aux_pre, int64_t ldc,
               int64_t n_store, int64_t ksplit, const OptT& bias_grad, int64_t defer) {
  const int64_t NS = (n_store <= 0 || n_store > N) ? N : n_store;
  CHECK_GPU(A, at::kBFloat16);
  CHECK_GPU(B, at::kBFloat16);
  if (mode == 0) {
    check_span(A, M, lda, K, "A");
    check_span(B, N, ldb, K, "B");
  } else if (mode == 1) {
    check_span(A, M, lda, K, "A");
    check_span(B, K, ldb, N, "B");
  } else {
    check_span(A, K, lda, M, "A");
    check_span(B, K, ldb, N, "B");
  }
  for (const OptT* o : {&resid, &out_f32}) {
    if (has(*o)) check_span(**o, M, ldc, NS, "out/resid");
  }
  for (const OptT* o : {&aux_in, &out_bf16, &aux_pre}) {
    if (has(*o)) check_span(**o, M, ldc, NS, "bf16 out/aux");
  }
  if (has(bias)) TORCH_CHECK(bias->numel() >= N, "bias too small");
  if (has(bias_grad)) TORCH_CHECK(bias_grad->numel() >= M, "bias_grad too small");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const int rc = mta_gemm_bf16((int)mode, A.data_ptr(), B.data_ptr(), (int)M, (int)N, (int)K, (int)lda, (int)ldb,
                               (float)alpha, (int)flags, opt_typed<float>(bias, at::kFloat, "bias"),
                               opt_typed<float>(resid, at::kFloat, "resid"),
                               opt_typed<void>(aux_in, at::kBFloat16, "aux_in"),
                               reinterpret_cast<const uint64_t*>(opt_typed<int64_t>(seed, at::kLong, "seed")),
                               (float)drop_p, opt_typed<void>(out_bf16, at::kBFloat16, "out_bf16"),
                               opt_typed<float>(out_f32, at::kFloat, "out_f32"),
                               opt_typed<void>(aux_pre, at::kBFloat16, "aux_pre"), (int)ldc, (int)NS, (int)ksplit,
                               opt_typed<float>(bias_grad, at::kFloat, "bias_grad"), (int)defer, cur_stream());
  TORCH_CHECK(rc == 0, "gemm_bf16: unsupported arguments (rc=", rc, ", M=", M, " N=", N, " K=", K, ")");
}

void cast_pad(std::vector<at::Tensor> src, std::vector<at::Tensor> dst, const OptT& seeds) {
  TORCH_CHECK(src.size() == dst.size() && !src.empty() && src.size() <= 16, "cast_pad: 1..16 tensor pairs");
  std::vector<const float*> sp;
  std::vector<void*> dp;
  std::vector<int> rows, cols, rows_p, cols_p, ld;
  for (size_t i = 0; i < src.size(); ++i) {
    auto s2 = src[i].dim() == 1 ? src[i].view({1, -1}) : src[i];
    auto d2 = dst[i].dim() == 1 ? dst[i].view({1, -1}) : dst[i];
    TORCH_CHECK(s2.dim() == 2 && d2.dim() == 2, "cast_pad: 1-D or 2-D tensors");
    TORCH_CHECK(s2.is_cuda() && s2.scalar_type() == at::kFloat && s2.stride(1) == 1, "cast_pad: src fp32 rows");
    CHECK_GPU(d2, at::kBFloat16);
    TORCH_CHECK(d2.size(0) >= s2.size(0) && d2.size(1) >= s2.size(1), "cast_pad: dst smaller than src");
    sp.push_back(s2.data_ptr<float>());
    dp.push_back(d2.data_ptr());
    rows.push_back((int)s2.size(0));
    cols.push_back((int)s2.size(1));
    rows_p.push_back((int)d2.size(0));
    cols_p.push_back((int)d2.size(1));
    ld.push_back((int)s2.stride(0));
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(src[0].device());
  uint64_t* sd = nullptr;
  int ns = 0;
  if (seeds.has_value() && seeds->defined()) {
    CHECK_GPU(*seeds, at::kLong);
    sd = reinterpret_cast<uint64_t*>(seeds->data_ptr<int64_t>());
    ns = (int)seeds->numel();
  }
  TORCH_CHECK(mta_cast_pad((int)src.size(), sp.data(), dp.data(), rows.data(), cols.data(), rows_p.data(),
                           cols_p.data(), ld.data(), sd, ns, cur_stream()) == 0, "cast_pad failed");
}

void norm(bool bwd, at::Tensor x, int64_t ldx, int64_t M, int64_t D, bool rms, double eps, const OptT& gamma,
          const OptT& beta, const OptT& y_bf16, const OptT& y_f32, const OptT& mean, at::Tensor rstd,
          const OptT& seed, double drop_p, const OptT& dy, const OptT& dres, const OptT& pre, const OptT& dx_bf16,
          const OptT& dx_f32, const OptT& dgamma, const OptT& dbeta, bool gelu_x, const OptT& hw_a,
          const OptT& hb_a, const OptT& hw_b, const OptT& hb_b, const OptT& ab, int64_t ab_rows, const OptT& g_wa,
          const OptT& g_wb) {
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "x must be fp32 or bf16 GPU");
  const bool xb = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(!gelu_x || xb, "gelu_x: x is the bf16 GELU input");
  if (has(ab)) {
    TORCH_CHECK(ab->is_contiguous() && ab->numel() >= 2 * (bwd ? ab_rows : M), "ab: contiguous (rows, 2) fp32");
    for (const OptT* o : {&hw_a, &hw_b}) TORCH_CHECK(has(*o) && (*o)->numel() >= D, "fused heads: (1, D) weights");
    if (bwd) TORCH_CHECK(has(g_wa) && has(g_wb) && g_wa->numel() >= D && g_wb->numel() >= D, "head-weight grads");
  }
  const bool dyb = has(dy) && dy->scalar_type() == at::kBFloat16;
  const bool pre_f = has(pre) && pre->scalar_type() == at::kFloat;  // fp32 GELU input (32-true extras)
  if (dyb) TORCH_CHECK(dy->is_cuda() && dy->is_contiguous(), "dy: contiguous GPU tensor");
  check_span(x, M, ldx, D, "x");
  CHECK_F32(rstd);
  TORCH_CHECK(rstd.numel() >= M, "rstd too small");
  if (!rms) TORCH_CHECK(has(mean) && mean->numel() >= M, "LayerNorm needs mean");
  if (bwd) TORCH_CHECK(has(dy) || has(ab), "norm backward needs dy (or the fused heads' d(alpha, beta))");
  for (const OptT* o : {&y_bf16, &y_f32, &dy, &pre}) {
    if (has(*o)) check_span(**o, M, D, D, "row tensor");
  }
  for (const OptT* o : {&dres, &dx_f32, &dx_bf16}) {
    if (has(*o)) check_span(**o, M, ldx, D, "residual-stride tensor");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int rc = mta_norm(bwd ? 1 : 0, x.data_ptr(), gelu_x ? 2 : xb ? 1 : 0, (int)ldx, (int)M, (int)D, rms ? 1 : 0, (float)eps,
                          opt_typed<float>(gamma, at::kFloat, "gamma"), opt_typed<float>(beta, at::kFloat, "beta"),
                          opt_typed<void>(y_bf16, at::kBFloat16, "y_bf16"), opt_typed<float>(y_f32, at::kFloat, "y_f32"),
                          opt_typed<float>(mean, at::kFloat, "mean"), rstd.data_ptr<float>(),
                          reinterpret_cast<const uint64_t*>(opt_typed<int64_t>(seed, at::kLong, "seed")),
                          (float)drop_p, dyb ? dy->data_ptr() : (const void*)opt_typed<float>(dy, at::kFloat, "dy"),
                          dyb ? 1 : 0,
                          opt_typed<float>(dres, at::kFloat, "dres"),
                          pre_f ? (const void*)opt_typed<float>(pre, at::kFloat, "pre")
                                : (const void*)opt_typed<void>(pre, at::kBFloat16, "pre"),
                          pre_f ? 1 : 0,
                          opt_typed<void>(dx_bf16, at::kBFloat16, "dx_bf16"),
                          opt_typed<float>(dx_f32, at::kFloat, "dx_f32"), opt_typed<float>(dgamma, at::kFloat, "dgamma"),
                          opt_typed<float>(dbeta, at::kFloat, "dbeta"), opt_typed<float>(hw_a, at::kFloat, "hw_a"),
                          opt_typed<float>(hb_a, at::kFloat, "hb_a"), opt_typed<float>(hw_b, at::kFloat, "hw_b"),
                          opt_typed<float>(hb_b, at::kFloat, "hb_b"), opt_typed<float>(ab, at::kFloat, "ab"),
                          (int)ab_rows, opt_typed<float>(g_wa, at::kFloat, "g_wa"),
                          opt_typed<float>(g_wb, at::kFloat, "g_wb"), cur_stream());
  TORCH_CHECK(rc == 0, "norm: unsupported arguments (D=", D, ", rc=", rc, ")");
}

// RoPE (cos, sin) table [T][HD/2] in fp64 -> fp32, built once per (device, T, HD, base) on the first (eager) call;
// graph replays reuse the cached device tensor
static const float* rope_table(const at::Device& dev, int64_t T, int64_t HD, double base) {
  static std::map<std::tuple<int, int64_t, int64_t, double>, at::Tensor> cache;
  const auto key = std::make_tuple((int)dev.index(), T, HD, base);
  auto it = cache.find(key);
  if (it == cache.end()) {
    auto host = at::empty({T * HD}, at::TensorOptions().dtype(at::kFloat));
    float* h = host.data_ptr<float>();
    for (int64_t t = 0; t < T; ++t)
      for (int64_t i = 0; i < HD / 2; ++i) {
        const double ang = (double)t * std::pow(base, -2.0 * (double)i / (double)HD);
        h[(t * (HD / 2) + i) * 2] = (float)std::cos(ang);
        h[(t * (HD / 2) + i) * 2 + 1] = (float)std::sin(ang);
      }
    it = cache.emplace(key, host.to(dev)).first;
  }
  return it->second.data_ptr<float>();
}

// optional bf16 [rows][cols] operand of the fused FFN (nullptr when absent)
void* opt_bf16(const OptT& t, int64_t numel, const char* name) {
  if (!has(t)) return nullptr;
  CHECK_GPU(*t, at::kBFloat16);
  TORCH_CHECK(t->numel() >= numel, name, ": too small");
  return t->data_ptr();
}

// fused FFN half of a transformer block (csrc/tr_ffn.hip), forward: x1 -> xn2, r2, pre, u, x2.
// xn2 / u (row-major) and xn2T / uT ([features][M], the k-contiguous weight-gradient operands) are each optional.
void tr_ffn_fwd(at::Tensor x1, at::Tensor w1, at::Tensor w2, at::Tensor b1, at::Tensor b2, at::Tensor g2, double eps,
                const OptT& seed, double drop_p, const OptT& xn2, at::Tensor r2, at::Tensor pre, const OptT& u,
                at::Tensor x2, const OptT& xn2T, const OptT& uT) {
  const int64_t d = x1.size(-1), M = x1.numel() / d, dff = w1.size(0);
  CHECK_F32(x1);
  CHECK_F32(x2);
  CHECK_F32(r2);
  for (auto* t : {&w1, &w2, &pre}) {
    CHECK_GPU(*t, at::kBFloat16);
  }
  TORCH_CHECK(w1.size(1) == d && w2.size(0) == d && w2.size(1) == dff, "tr_ffn_fwd: weight shapes");
  TORCH_CHECK(x2.numel() >= M * d && pre.numel() >= M * dff && r2.numel() >= M && b1.numel() >= dff &&
                  b2.numel() >= d && g2.numel() >= d,
              "tr_ffn_fwd: sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x1.device());
  const int rc = mta_tr_ffn(0, (int)M, (int)d, (int)dff, (float)eps, w1.data_ptr(), w2.data_ptr(), b1.data_ptr<float>(),
                            b2.data_ptr<float>(), g2.data_ptr<float>(), x1.data_ptr<float>(),
                            reinterpret_cast<const uint64_t*>(opt_typed<int64_t>(seed, at::kLong, "seed")),
                            (float)drop_p, opt_bf16(xn2, M * d, "xn2"), pre.data_ptr(), opt_bf16(u, M * dff, "u"),
                            r2.data_ptr<float>(), x2.data_ptr<float>(), nullptr, nullptr, nullptr, nullptr, nullptr,
                            nullptr, nullptr, nullptr, opt_bf16(uT, M * dff, "uT"), opt_bf16(xn2T, M * d, "xn2T"),
                            nullptr, nullptr, cur_stream());
  TORCH_CHECK(rc == 0, "tr_ffn_fwd: unsupported configuration (d=", d, ", dff=", dff, ", rc=", rc, ")");
}

// backward (input gradients): dX (fp32 + its bf16 copy) -> dpre (bf16), dX1 (fp32 + bf16), dg2 +=
// w1t = W1^T [d][dff], w2t = W2^T [dff][d]; dpre row-major and dpreT / dxT ([features][M]) are each optional
void tr_ffn_bwd(at::Tensor x1, at::Tensor w1t, at::Tensor w2t, at::Tensor g2, at::Tensor r2, at::Tensor pre,
                const OptT& seed, double drop_p, at::Tensor dx, at::Tensor dxb, const OptT& dpre, at::Tensor dx1,
                at::Tensor dx1b, at::Tensor dg2, const OptT& dpreT, const OptT& dxT) {
  const int64_t d = x1.size(-1), M = x1.numel() / d, dff = w1t.size(1);
  for (auto* t : {&x1, &r2, &dx, &dx1, &dg2}) {
    CHECK_F32(*t);
  }
  for (auto* t : {&w1t, &w2t, &pre, &dxb, &dx1b}) {
    CHECK_GPU(*t, at::kBFloat16);
  }
  TORCH_CHECK(w1t.size(0) == d && w2t.size(0) == dff && w2t.size(1) == d, "tr_ffn_bwd: weight shapes");
  TORCH_CHECK(dx.numel() >= M * d && dxb.numel() >= M * d && dx1.numel() >= M * d && dx1b.numel() >= M * d &&
                  pre.numel() >= M * dff && r2.numel() >= M && dg2.numel() >= d,
              "tr_ffn_bwd: sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x1.device());
  const int rc = mta_tr_ffn(1, (int)M, (int)d, (int)dff, 0.f, w1t.data_ptr(), w2t.data_ptr(), nullptr, nullptr,
                            g2.data_ptr<float>(), x1.data_ptr<float>(),
                            reinterpret_cast<const uint64_t*>(opt_typed<int64_t>(seed, at::kLong, "seed")),
                            (float)drop_p, nullptr, nullptr, nullptr, nullptr, nullptr, dxb.data_ptr(),
                            dx.data_ptr<float>(), r2.data_ptr<float>(), pre.data_ptr(), opt_bf16(dpre, M * dff, "dpre"),
                            dx1.data_ptr<float>(), dx1b.data_ptr(), dg2.data_ptr<float>(), nullptr, nullptr,
                            opt_bf16(dpreT, M * dff, "dpreT"), opt_bf16(dxT, M * d, "dxT"), cur_stream());
  TORCH_CHECK(rc == 0, "tr_ffn_bwd: unsupported configuration (d=", d, ", dff=", dff, ", rc=", rc, ")");
}

// fp32 matrices -> bf16 fragment-major [N][K] images (csrc/tr_ffn.hip): src [N][K], or with transposed[i] src [K][N]
// and image(n, k) = src[k][n] -- the fused transformer halves' weights, every layer in one launch
void frag_pack(std::vector<at::Tensor> src, std::vector<at::Tensor> dst, std::vector<bool> transposed,
               std::vector<at::Tensor> cast_src, std::vector<at::Tensor> cast_dst, const OptT& seeds) {
  TORCH_CHECK(!src.empty() && src.size() == dst.size() && src.size() == transposed.size() && src.size() <= 32,
              "frag_pack: 1..32 matrices");
  TORCH_CHECK(cast_src.size() == cast_dst.size() && cast_src.size() <= 4, "frag_pack: at most 4 riding casts");
  std::vector<const float*> sp;
  std::vector<void*> dp;
  std::vector<int> n, k, tr;
  for (size_t i = 0; i < src.size(); ++i) {
    CHECK_F32(src[i]);
    CHECK_GPU(dst[i], at::kBFloat16);
    TORCH_CHECK(src[i].dim() == 2 && dst[i].numel() == src[i].numel(), "frag_pack: shapes");
    sp.push_back(src[i].data_ptr<float>());
    dp.push_back(dst[i].data_ptr());
    n.push_back((int)src[i].size(transposed[i] ? 1 : 0));
    k.push_back((int)src[i].size(transposed[i] ? 0 : 1));
    tr.push_back(transposed[i] ? 1 : 0);
  }
  // riding casts: the cast_pad contract (fp32 rows -> zero-padded bf16)
  std::vector<const float*> csp;
  std::vector<void*> cdp;
  std::vector<int> rows, cols, rows_p, cols_p, ld;
  for (size_t i = 0; i < cast_src.size(); ++i) {
    auto s2 = cast_src[i].dim() == 1 ? cast_src[i].view({1, -1}) : cast_src[i];
    auto d2 = cast_dst[i].dim() == 1 ? cast_dst[i].view({1, -1}) : cast_dst[i];
    TORCH_CHECK(s2.dim() == 2 && d2.dim() == 2, "frag_pack casts: 1-D or 2-D tensors");
    TORCH_CHECK(s2.is_cuda() && s2.scalar_type() == at::kFloat && s2.stride(1) == 1, "frag_pack casts: src fp32 rows");
    CHECK_GPU(d2, at::kBFloat16);
    TORCH_CHECK(d2.size(0) >= s2.size(0) && d2.size(1) >= s2.size(1), "frag_pack casts: dst smaller than src");
    csp.push_back(s2.data_ptr<float>());
    cdp.push_back(d2.data_ptr());
    rows.push_back((int)s2.size(0));
    cols.push_back((int)s2.size(1));
    rows_p.push_back((int)d2.size(0));
    cols_p.push_back((int)d2.size(1));
    ld.push_back((int)s2.stride(0));
  }
  uint64_t* sd = nullptr;
  int ns = 0;
  if (seeds.has_value() && seeds->defined()) {
    CHECK_GPU(*seeds, at::kLong);
    sd = reinterpret_cast<uint64_t*>(seeds->data_ptr<int64_t>());
    ns = (int)seeds->numel();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dst[0].device());
  const int rc = mta_frag_pack((int)sp.size(), sp.data(), dp.data(), n.data(), k.data(), tr.data(), (int)csp.size(),
                               csp.data(), cdp.data(), rows.data(), cols.data(), rows_p.data(), cols_p.data(),
                               ld.data(), sd, ns, cur_stream());
  TORCH_CHECK(rc == 0, "frag_pack: N must be a multiple of 16 and K of 32 (rc=", rc, ")");
}

// backward tail of the fused attention half (csrc/tr_attn.hip tr_attn_dx_kernel): d(xn) = dqkv Wqkv, RMSNorm1
// backward + residual -> dx (fp32), dxb (bf16); dg1 through a deferred norm slot (summed at norm_flush)
void tr_attn_dx(at::Tensor dqkv, at::Tensor wqkvt, at::Tensor x, at::Tensor r1, at::Tensor g1, at::Tensor dx1,
                at::Tensor dx, at::Tensor dxb, at::Tensor dg1) {
  CHECK_GPU(dqkv, at::kBFloat16);
  CHECK_GPU(wqkvt, at::kBFloat16);
  CHECK_GPU(dxb, at::kBFloat16);
  for (auto* t : {&x, &r1, &g1, &dx1, &dx, &dg1}) {
    CHECK_F32(*t);
  }
  const int64_t M = x.size(0);
  TORCH_CHECK(x.dim() == 2 && x.size(1) == 128 && dx1.numel() == M * 128 && dx.numel() == M * 128 &&
                  dxb.numel() == M * 128 && dqkv.numel() == M * 384 && r1.numel() >= M && g1.numel() == 128 &&
                  dg1.numel() == 128 && wqkvt.numel() == 128 * 384,
              "tr_attn_dx: d = 128, 4 heads (dqkv [M][384], x / dx1 / dx [M][128])");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int rc = mta_tr_attn_dx((int)M, dqkv.data_ptr(), wqkvt.data_ptr(), x.data_ptr<float>(), r1.data_ptr<float>(),
                                g1.data_ptr<float>(), dx1.data_ptr<float>(), dx.data_ptr<float>(), dxb.data_ptr(),
                                dg1.data_ptr<float>(), cur_stream());
  TORCH_CHECK(rc == 0, "tr_attn_dx failed (rc=", rc, ")");
}

// fused attention half of a transformer block forward (csrc/tr_attn.hip): x -> xn, r1, qkv, o, lse, x1
void tr_attn_fwd(int64_t nseq, int64_t T, int64_t heads, double eps, double rope_base, at::Tensor x, at::Tensor wqkv,
                 at::Tensor wo, at::Tensor g1, at::Tensor bqkv, at::Tensor bo, at::Tensor xn, at::Tensor r1,
                 at::Tensor qkv, at::Tensor o, at::Tensor lse, at::Tensor x1, const OptT& in, const OptT& we,
                 const OptT& be) {
  // in / we / be given: the block input x = in We^T + be is computed in the kernel (the embedding) and WRITTEN to x
  const int64_t d = x.size(-1), M = nseq * T;
  const bool emb = has(in);
  if (emb) {
    TORCH_CHECK(has(we) && has(be), "tr_attn_fwd: the embedding needs in, we and be");
    CHECK_F32(*in);
    CHECK_F32(*we);
    CHECK_F32(*be);
    TORCH_CHECK(in->dim() == 2 && in->size(1) <= 8 && we->size(0) == d && we->size(1) == in->size(1) &&
                    be->numel() == d && in->size(0) <= M,
                "tr_attn_fwd: embedding shapes (in [rows][F <= 8], we [d][F], be [d])");
  }
  for (auto* t : {&x, &r1, &lse, &x1, &g1, &bqkv, &bo}) {
    CHECK_F32(*t);
  }
  for (auto* t : {&wqkv, &wo, &xn, &qkv, &o}) {
    CHECK_GPU(*t, at::kBFloat16);
  }
  TORCH_CHECK(wqkv.size(0) == 3 * d && wqkv.size(1) == d && wo.size(0) == d && wo.size(1) == d,
              "tr_attn_fwd: weight shapes");
  TORCH_CHECK(x.numel() >= M * d && x1.numel() >= M * d && xn.numel() >= M * d && o.numel() >= M * d &&
                  qkv.numel() >= M * 3 * d && r1.numel() >= M && lse.numel() >= nseq * heads * 64,
              "tr_attn_fwd: sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int rc = mta_tr_attn_fwd((int)nseq, (int)T, (int)d, (int)heads, x.data_ptr<float>(), wqkv.data_ptr(),
                                 wo.data_ptr(), g1.data_ptr<float>(), bqkv.data_ptr<float>(), bo.data_ptr<float>(),
                                 rope_table(x.device(), T, d / heads, rope_base), (float)eps, xn.data_ptr(),
                                 r1.data_ptr<float>(), qkv.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                                 x1.data_ptr<float>(), emb ? in->data_ptr<float>() : nullptr,
                                 emb ? we->data_ptr<float>() : nullptr, emb ? be->data_ptr<float>() : nullptr,
                                 emb ? (int)in->size(1) : 0, emb ? (int)in->size(0) : 0,
                                 emb ? x.data_ptr<float>() : nullptr, cur_stream());
  TORCH_CHECK(rc == 0, "tr_attn_fwd: unsupported configuration (d=", d, ", heads=", heads, ", T=", T, ", rc=", rc, ")");
}

// dst[i] = src[i]^T for bf16 matrices (one launch)
void transpose_bf16(std::vector<at::Tensor> src, std::vector<at::Tensor> dst) {
  TORCH_CHECK(src.size() == dst.size() && !src.empty() && src.size() <= 32, "transpose_bf16: 1..32 matrices");
  std::vector<const void*> sp;
  std::vector<void*> dp;
  std::vector<int> rows, cols;
  for (size_t i = 0; i < src.size(); ++i) {
    CHECK_GPU(src[i], at::kBFloat16);
    CHECK_GPU(dst[i], at::kBFloat16);
    TORCH_CHECK(src[i].dim() == 2 && dst[i].dim() == 2 && dst[i].size(0) == src[i].size(1) &&
                    dst[i].size(1) == src[i].size(0) && src[i].is_contiguous() && dst[i].is_contiguous(),
                "transpose_bf16: dst must be the contiguous [cols][rows] of src");
    sp.push_back(src[i].data_ptr());
    dp.push_back(dst[i].data_ptr());
    rows.push_back((int)src[i].size(0));
    cols.push_back((int)src[i].size(1));
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(src[0].device());
  const int rc = mta_tr_transpose_bf16((int)sp.size(), sp.data(), dp.data(), rows.data(), cols.data(), cur_stream());
  TORCH_CHECK(rc == 0, "transpose_bf16: rows/cols must be multiples of 8 (rc=", rc, ")");
}

void attention(bool bwd, at::Tensor qkv, at::Tensor out, at::Tensor lse, const OptT& dout, const OptT& dqkv,
               int64_t nseq, int64_t T, int64_t D, int64_t heads, double rope_base, const OptT& dx1,
               const OptT& wot) {
  CHECK_GPU(qkv, at::kBFloat16);
  CHECK_GPU(out, at::kBFloat16);
  CHECK_F32(lse);
  TORCH_CHECK(qkv.numel() >= nseq * T * 3 * D && out.numel() >= nseq * T * D, "attention: qkv/out too small");
  TORCH_CHECK(lse.numel() >= nseq * heads * 64, "attention: lse must hold nseq*heads*64");
  if (bwd) {
    TORCH_CHECK(has(dqkv) && (has(dout) || (has(dx1) && has(wot))),
                "attention backward needs dqkv and dout (or dx1 + wot: the fused output-projection gradient)");
    TORCH_CHECK(dqkv->numel() >= nseq * T * 3 * D, "attention: dqkv too small");
    if (has(dout)) TORCH_CHECK(dout->numel() >= nseq * T * D, "attention: dout too small");
    if (has(dx1)) {
      CHECK_GPU(*dx1, at::kBFloat16);
      CHECK_GPU(*wot, at::kBFloat16);
      TORCH_CHECK(dx1->numel() >= nseq * T * D && wot->numel() >= D * D, "attention: dx1 / wot too small");
    }
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  const int rc = mta_attention(bwd ? 1 : 0, qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(),
                               opt_typed<void>(dout, at::kBFloat16, "dout"), opt_typed<void>(dqkv, at::kBFloat16, "dqkv"),
                               (int)nseq, (int)T, (int)D, (int)heads, (float)rope_base,
                               rope_table(qkv.device(), T, D / heads, rope_base),
                               has(dx1) ? dx1->data_ptr() : nullptr, has(wot) ? wot->data_ptr() : nullptr,
                               cur_stream());
  TORCH_CHECK(rc == 0, "attention: unsupported configuration (T=", T, ", D=", D, ", heads=", heads, ", rc=", rc, ")");
}


// fp32 RoPE attention of the 32-true transformer (csrc/attention_f32.hip): forward o, lse <- qkv; backward dqkv <-
// (qkv, o, dout, lse)
void attention_f32(bool bwd, at::Tensor qkv, at::Tensor out, at::Tensor lse, const OptT& dout, const OptT& dqkv,
                   int64_t nseq, int64_t T, int64_t D, int64_t heads, double rope_base) {
  CHECK_F32(qkv);
  CHECK_F32(out);
  CHECK_F32(lse);
  TORCH_CHECK(qkv.numel() >= nseq * T * 3 * D && out.numel() >= nseq * T * D, "attention_f32: qkv/out too small");
  TORCH_CHECK(lse.numel() >= nseq * heads * 64, "attention_f32: lse must hold nseq*heads*64");
  if (bwd) {
    TORCH_CHECK(has(dout) && has(dqkv), "attention_f32 backward needs dout and dqkv");
    CHECK_F32(*dout);
    CHECK_F32(*dqkv);
    TORCH_CHECK(dout->numel() >= nseq * T * D && dqkv->numel() >= nseq * T * 3 * D, "attention_f32: grads too small");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  const int rc = mta_attention_f32(bwd ? 1 : 0, qkv.data_ptr<float>(), bwd ? out.data_ptr<float>() : nullptr,
                                   bwd ? dout->data_ptr<float>() : nullptr, bwd ? nullptr : out.data_ptr<float>(),
                                   lse.data_ptr<float>(), bwd ? dqkv->data_ptr<float>() : nullptr, (int)nseq, (int)T,
                                   (int)D, (int)heads, rope_table(qkv.device(), T, D / heads, rope_base), cur_stream());
  TORCH_CHECK(rc == 0, "attention_f32: unsupported configuration (T=", T, ", D=", D, ", heads=", heads, ", rc=", rc,
              ")");
}

// ------------------------------------------------------------------------------- pipelined LSTM stack
// list entries with numel() == 0 stand for "no tensor"
std::vector<float*> ptrs_f32(const std::vector<at::Tensor>& v, const char* name) {
  std::vector<float*> out;
  for (const auto& t : v) {
    if (!t.defined() || t.numel() == 0) {
      out.push_back(nullptr);
      continue;
    }
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name, ": fp32 contiguous GPU");
    out.push_back(t.data_ptr<float>());
  }
  return out;
}

int64_t lstm_stack_flag_words(int64_t Np) { return mta_lstm_stack_flag_words((int)Np); }

static void lstm_stack_fwd_impl(int64_t H, int64_t prec, int64_t fin, at::Tensor x, std::vector<at::Tensor> w_ih,
                                std::vector<at::Tensor> w_hh, std::vector<at::Tensor> b_ih,
                                std::vector<at::Tensor> b_hh, std::vector<at::Tensor> hseq,
                                std::vector<at::Tensor> xdrop, std::vector<at::Tensor> masks,
                                std::vector<at::Tensor> stash, at::Tensor seeds, double drop_p, at::Tensor flags,
                                int64_t N, int64_t Np, int64_t T, const MtaBatchGather* gather, const OptT& gran) {
  const int64_t L = (int64_t)w_hh.size();
  // gran: the decoupled form's layer hand-off granules, int64[(L - 1) * T * Np * H] (L = 1: any, even empty);
  // None selects the barrier form (MTA_LSTM_DEC=0)
  const bool dec = has(gran);
  if (dec) {
    TORCH_CHECK(gran->is_cuda() && gran->scalar_type() == at::kLong && gran->numel() >= (L - 1) * T * Np * H,
                "gran: int64[(L - 1) * T * Np * H] hand-off granules");
  }
  CHECK_F32(x);
  TORCH_CHECK(x.numel() == N * T * fin, "x must be (N, T, F)");
  TORCH_CHECK(w_ih.size() == (size_t)L && b_ih.size() == (size_t)L && b_hh.size() == (size_t)L &&
              hseq.size() == (size_t)L && xdrop.size() == (size_t)L && stash.size() == (size_t)L, "per-layer lists");
  for (int64_t l = 0; l < L; ++l) {
    TORCH_CHECK(w_hh[l].numel() == 4 * H * H && w_ih[l].numel() == 4 * H * (l == 0 ? fin : H), "weight shapes");
    TORCH_CHECK(hseq[l].numel() == T * Np * H, "hseq shape");
    if (xdrop[l].numel()) TORCH_CHECK(l > 0 && xdrop[l].numel() == T * Np * H, "xdrop shape");
    TORCH_CHECK(masks.size() == (size_t)L, "per-layer keep-byte list");
    if (xdrop[l].numel())
      TORCH_CHECK(masks[l].is_cuda() && masks[l].scalar_type() == at::kByte && masks[l].numel() == T * Np * H,
                  "keep bytes: uint8[T * Np * H] per dropout layer (u32 words (T, ntiles, 4, H))");
    if (stash[l].numel()) TORCH_CHECK(stash[l].numel() == T * Np * 5 * H, "stash shape");
  }
  TORCH_CHECK(seeds.is_cuda() && seeds.scalar_type() == at::kLong && seeds.numel() >= L, "seeds: int64[L]");
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kInt && flags.numel() >= lstm_stack_flag_words(Np),
              "flags: int32 scratch of lstm_stack_flag_words(Np)");
  auto wi = ptrs_f32(w_ih, "w_ih"), wh = ptrs_f32(w_hh, "w_hh"), bi = ptrs_f32(b_ih, "b_ih"),
       bh = ptrs_f32(b_hh, "b_hh"), hs = ptrs_f32(hseq, "hseq"), xd = ptrs_f32(xdrop, "xdrop"),
       sh = ptrs_f32(stash, "stash");
  std::vector<const float*> cwi(wi.begin(), wi.end()), cwh(wh.begin(), wh.end()), cbi(bi.begin(), bi.end()),
      cbh(bh.begin(), bh.end());
  std::vector<uint32_t*> mk(L, nullptr);
  for (int64_t l = 0; l < L; ++l)
    if (xdrop[l].numel()) mk[l] = reinterpret_cast<uint32_t*>(masks[l].data_ptr<uint8_t>());
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int rc = mta_lstm_stack_fwd_g((int)H, (int)prec, (int)L, (int)fin, x.data_ptr<float>(), cwi.data(),
                                      cwh.data(), cbi.data(), cbh.data(), hs.data(), xd.data(), mk.data(), sh.data(),
                                      reinterpret_cast<const uint64_t*>(seeds.data_ptr<int64_t>()), (float)drop_p,
                                      reinterpret_cast<unsigned*>(flags.data_ptr<int>()), (int)N, (int)Np, (int)T,
                                      gather,
                                      dec && L > 1 ? reinterpret_cast<unsigned long long*>(gran->data_ptr<int64_t>())
                                                   : nullptr,
                                      dec ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "lstm_stack_fwd: unsupported configuration (rc=", rc, ")");
}

void lstm_stack_fwd(int64_t H, int64_t prec, int64_t fin, at::Tensor x, std::vector<at::Tensor> w_ih,
                    std::vector<at::Tensor> w_hh, std::vector<at::Tensor> b_ih, std::vector<at::Tensor> b_hh,
                    std::vector<at::Tensor> hseq, std::vector<at::Tensor> xdrop, std::vector<at::Tensor> masks,
                    std::vector<at::Tensor> stash, at::Tensor seeds, double drop_p, at::Tensor flags, int64_t N,
                    int64_t Np, int64_t T, const OptT& gran) {
  lstm_stack_fwd_impl(H, prec, fin, x, w_ih, w_hh, b_ih, b_hh, hseq, xdrop, masks, stash, seeds, drop_p, flags, N, Np,
                      T, nullptr, gran);
}

// the same launch with the training step's batch gather folded in: src[k] (rows, ...) -> dst[k] (B, ...) at rows
// perm[cursor * B + b]; x must be dst[0] (the static batch buffer), cursor advances once per launch
void lstm_stack_fwd_gather(int64_t H, int64_t prec, int64_t fin, at::Tensor x, std::vector<at::Tensor> w_ih,
                           std::vector<at::Tensor> w_hh, std::vector<at::Tensor> b_ih, std::vector<at::Tensor> b_hh,
                           std::vector<at::Tensor> hseq, std::vector<at::Tensor> xdrop,
                           std::vector<at::Tensor> masks, std::vector<at::Tensor> stash, at::Tensor seeds,
                           double drop_p, at::Tensor flags, int64_t N, int64_t Np, int64_t T,
                           std::vector<at::Tensor> src, std::vector<at::Tensor> dst, at::Tensor perm, at::Tensor cursor,
                           int64_t B, const OptT& gran) {
  TORCH_CHECK(src.size() == dst.size() && src.size() >= 1 && src.size() <= 4, "1..4 gathered tensors");
  TORCH_CHECK(perm.is_cuda() && cursor.is_cuda() && perm.scalar_type() == at::kInt &&
              cursor.scalar_type() == at::kInt, "perm/cursor: int32 GPU tensors");
  TORCH_CHECK(dst[0].data_ptr() == x.data_ptr(), "x must be the static batch buffer dst[0]");
  MtaBatchGather g{};
  for (size_t k = 0; k < src.size(); ++k) {
    CHECK_F32(src[k]);
    CHECK_F32(dst[k]);
    g.row[k] = (long)(src[k].numel() / src[k].size(0));
    TORCH_CHECK(dst[k].numel() == B * g.row[k], "dst ", k, " must hold B rows");
    g.src[k] = src[k].data_ptr<float>();
    g.dst[k] = dst[k].data_ptr<float>();
  }
  g.nt = (int)src.size();
  g.perm = perm.data_ptr<int>();
  g.cursor = cursor.data_ptr<int>();
  g.B = (int)B;
  lstm_stack_fwd_impl(H, prec, fin, x, w_ih, w_hh, b_ih, b_hh, hseq, xdrop, masks, stash, seeds, drop_p, flags, N, Np,
                      T, &g, gran);
}

// grads: [] (weight gradients by the caller) or 4 lists g_wih, g_whh, g_bih, g_bhh of per-layer gradient
// views the fused weight-gradient workgroups accumulate into; inp[0] = x (N, T, fin), inp[l] = layer input.
void lstm_stack_bwd(int64_t H, int64_t prec, int64_t fin, std::vector<at::Tensor> stash, std::vector<at::Tensor> w_hh,
                    std::vector<at::Tensor> w_ih, at::Tensor dh_last, std::vector<at::Tensor> dG,
                    std::vector<at::Tensor> dX, std::vector<at::Tensor> hseq, std::vector<at::Tensor> inp,
                    std::vector<std::vector<at::Tensor>> grads, std::vector<at::Tensor> masks,
                    std::vector<at::Tensor> parts, at::Tensor seeds, double drop_p, bool dropout, at::Tensor flags,
                    int64_t N, int64_t Np, int64_t T, int64_t form) {
  // form: the dX hand-off, 0 = fp32 rows + progress words (the only form kept)
  TORCH_CHECK(form == 0, "form: 0 (fp32 rows + progress words)");
  const bool gran = false;
  const int64_t L = (int64_t)w_hh.size();
  CHECK_F32(dh_last);
  TORCH_CHECK(dh_last.numel() == N * H, "dh_last must be (N, H)");
  TORCH_CHECK(stash.size() == (size_t)L && w_ih.size() == (size_t)L && dG.size() == (size_t)L &&
              dX.size() == (size_t)L, "per-layer lists");
  for (int64_t l = 0; l < L; ++l) {
    TORCH_CHECK(stash[l].numel() == T * Np * 5 * H && dG[l].numel() == T * Np * 4 * H, "stash/dG shapes");
    TORCH_CHECK(l == L - 1 || dX[l].numel() == (gran ? 2 : 1) * T * Np * H, "dX shape");
  }
  const bool fused = !grads.empty();
  if (fused) {
    TORCH_CHECK(grads.size() == 4 && hseq.size() == (size_t)L && inp.size() == (size_t)L, "fused wgrad lists");
    for (int64_t l = 0; l < L; ++l) {
      const int64_t F = l == 0 ? fin : H;
      TORCH_CHECK(hseq[l].numel() == T * Np * H, "hseq shape");
      TORCH_CHECK(inp[l].numel() == (l == 0 ? N * T * fin : T * Np * H), "layer input shape");
      TORCH_CHECK(grads[0][l].numel() == 4 * H * F && grads[1][l].numel() == 4 * H * H &&
                      grads[2][l].numel() == 4 * H && grads[3][l].numel() == 4 * H,
                  "gradient view shapes");
    }
  }
  TORCH_CHECK(seeds.is_cuda() && seeds.scalar_type() == at::kLong && seeds.numel() >= L, "seeds: int64[L]");
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kInt && flags.numel() >= lstm_stack_flag_words(Np),
              "flags scratch too small");
  auto st = ptrs_f32(stash, "stash"), wh = ptrs_f32(w_hh, "w_hh"), wi = ptrs_f32(w_ih, "w_ih"),
       dg = ptrs_f32(dG, "dG"), dx = ptrs_f32(dX, "dX");
  std::vector<float*> hs, in, g0, g1, g2, g3;
  if (fused) {
    hs = ptrs_f32(hseq, "hseq");
    in = ptrs_f32(inp, "inp");
    g0 = ptrs_f32(grads[0], "g_wih");
    g1 = ptrs_f32(grads[1], "g_whh");
    g2 = ptrs_f32(grads[2], "g_bih");
    g3 = ptrs_f32(grads[3], "g_bhh");
  }
  std::vector<const float*> cst(st.begin(), st.end()), cwh(wh.begin(), wh.end()), cwi(wi.begin(), wi.end()),
      chs(hs.begin(), hs.end()), cin(in.begin(), in.end());
  std::vector<const uint32_t*> mk(L, nullptr);
  if (dropout) {
    TORCH_CHECK(masks.size() == (size_t)L, "per-layer keep-byte list");
    for (int64_t l = 1; l < L; ++l) {
      TORCH_CHECK(masks[l].is_cuda() && masks[l].scalar_type() == at::kByte && masks[l].numel() == T * Np * H,
                  "keep bytes: uint8[T * Np * H] per dropout layer (u32 words (T, ntiles, 4, H))");
      mk[l] = reinterpret_cast<const uint32_t*>(masks[l].data_ptr<uint8_t>());
    }
  }
  // deterministic mode: per-layer partial buffers of mta_lstm_wgrad_part_floats(1, T, H, F) floats
  std::vector<float*> pt;
  if (!parts.empty()) {
    TORCH_CHECK(fused && parts.size() == (size_t)L, "parts: one buffer per layer (fused weight gradients)");
    for (int64_t l = 0; l < L; ++l) {
      CHECK_F32(parts[l]);
      TORCH_CHECK(parts[l].numel() >= mta_lstm_wgrad_part_floats(1, (int)T, (int)H, l == 0 ? (int)fin : (int)H),
                  "parts buffer too small");
      pt.push_back(parts[l].data_ptr<float>());
    }
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dh_last.device());
  const int rc = mta_lstm_stack_bwd(
      (int)H, (int)prec, (int)L, (int)fin, cst.data(), cwh.data(), cwi.data(), dh_last.data_ptr<float>(), dg.data(),
      dx.data(), fused ? chs.data() : nullptr, fused ? cin.data() : nullptr, fused ? g0.data() : nullptr,
      fused ? g1.data() : nullptr, fused ? g2.data() : nullptr, fused ? g3.data() : nullptr, mk.data(),
      pt.empty() ? nullptr : pt.data(),
      reinterpret_cast<uint64_t*>(seeds.data_ptr<int64_t>()), (float)drop_p, dropout ? 1 : 0,
      reinterpret_cast<unsigned*>(flags.data_ptr<int>()), (int)N, (int)Np, (int)T, (int)form, cur_stream());
  TORCH_CHECK(rc == 0, "lstm_stack_bwd: unsupported configuration (rc=", rc, ")");
}


// ------------------------------------------------------------------------------- xGMI all-reduce
int64_t xgmi_buffer_bytes(int64_t world, int64_t cap, int64_t channels) {
  return (int64_t)mta_xgmi_buffer_bytes((int)world, (long)cap, (int)channels);
}

int64_t xgmi_alloc(int64_t bytes) {
  void* p = nullptr;
  const int rc = mta_xgmi_alloc((long)bytes, &p);
  TORCH_CHECK(rc == 0, "xgmi_alloc: fine-grained allocation failed (rc=", rc, ")");
  return reinterpret_cast<int64_t>(p);
}

void xgmi_free(int64_t p) { mta_xgmi_free(reinterpret_cast<void*>(p)); }

at::Tensor xgmi_ipc_handle(int64_t p) {
  at::Tensor out = at::zeros({64}, at::TensorOptions().dtype(at::kByte));
  const int n = mta_xgmi_ipc_handle(reinterpret_cast<void*>(p), out.data_ptr<uint8_t>());
  TORCH_CHECK(n > 0, "hipIpcGetMemHandle failed");
  return out;
}

int64_t xgmi_ipc_open(at::Tensor handle) {
  TORCH_CHECK(handle.scalar_type() == at::kByte && handle.numel() == 64 && !handle.is_cuda(), "64-byte CPU handle");
  void* p = nullptr;
  TORCH_CHECK(mta_xgmi_ipc_open(handle.contiguous().data_ptr<uint8_t>(), &p) == 0, "hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

void xgmi_ipc_close(int64_t p) { mta_xgmi_ipc_close(reinterpret_cast<void*>(p)); }

// in-place sum of `grad` (a bucket at flat offset `off` of the gradient) over the ranks on the current stream;
// bufs: every rank's comm buffer as mapped in this process; ctl: int32[xgmi_ctl_words] zero-initialised once
// (per-channel epoch and arrival counters, the shared timeout count)
void xgmi_allreduce(at::Tensor grad, int64_t off, int64_t cap, int64_t channel, int64_t channels, bool twoshot,
                    std::vector<int64_t> bufs, int64_t rank, at::Tensor ctl, const OptT& sq) {
  CHECK_F32(grad);
  TORCH_CHECK(ctl.is_cuda() && ctl.scalar_type() == at::kInt && ctl.numel() >= mta_xgmi_ctl_words(), "ctl words");
  if (has(sq)) {
    CHECK_F32(*sq);
    TORCH_CHECK(sq->numel() >= mta_xgmi_max_blocks(), "sq: xgmi_max_blocks() floats of clip-norm partials");
  }
  std::vector<void*> b;
  for (auto v : bufs) b.push_back(reinterpret_cast<void*>(v));
  c10::hip::HIPGuardMasqueradingAsCUDA guard(grad.device());
  const int rc = mta_xgmi_allreduce(grad.data_ptr<float>(), (long)grad.numel(), (long)off, (long)cap, (int)channel,
                                    (int)channels, twoshot ? 1 : 0, b.data(), (int)rank, (int)b.size(),
                                    reinterpret_cast<unsigned*>(ctl.data_ptr<int>()),
                                    has(sq) ? sq->data_ptr<float>() : nullptr, cur_stream());
  TORCH_CHECK(rc == 0, "xgmi_allreduce: bad arguments (rc=", rc, ")");
}

// ------------------------------------------------------------------------------- dataset build
void dgp(int64_t seed, int64_t mkt_df, double mkt_loc, double mkt_scale, int64_t idio_df, double idio_loc,
         double idio_scale, double a_loc, double a_scale, double b_loc, double b_scale, at::Tensor r_market,
         at::Tensor r_stocks, at::Tensor alphas, at::Tensor betas) {
  CHECK_F32(r_market);
  CHECK_F32(r_stocks);
  CHECK_F32(alphas);
  CHECK_F32(betas);
  const int64_t K = r_stocks.size(0), S = r_market.numel();
  TORCH_CHECK(r_stocks.dim() == 2 && r_stocks.size(1) == S && alphas.numel() == K && betas.numel() == K,
              "dgp: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(r_market.device());
  const int rc = mta_dgp((uint64_t)seed, (int)K, (long)S, (int)mkt_df, (float)mkt_loc, (float)mkt_scale,
                         (int)idio_df, (float)idio_loc, (float)idio_scale, (float)a_loc, (float)a_scale,
                         (float)b_loc, (float)b_scale, r_market.data_ptr<float>(), r_stocks.data_ptr<float>(),
                         alphas.data_ptr<float>(), betas.data_ptr<float>(), cur_stream());
  TORCH_CHECK(rc == 0, "dgp: unsupported degrees of freedom or sample count");
}

void ols_features(at::Tensor target, at::Tensor alphas, at::Tensor betas, at::Tensor factor, at::Tensor inv_psi) {
  CHECK_F32(target);
  TORCH_CHECK(target.dim() == 4 && target.size(3) >= 2 && target.size(2) >= 2, "target must be (W, K, n, C>=2)");
  const int64_t W = target.size(0), K = target.size(1);
  for (auto* t : {&alphas, &betas, &inv_psi}) {
    CHECK_F32(*t);
    TORCH_CHECK(t->numel() == W * K, "per-(window, stock) output shape");
  }
  CHECK_F32(factor);
  TORCH_CHECK(factor.numel() == W * 2, "factor must be (W, 2)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(target.device());
  mta_ols_features(target.data_ptr<float>(), (int)W, (int)K, (int)target.size(2), (int)target.size(3),
                   alphas.data_ptr<float>(), betas.data_ptr<float>(), factor.data_ptr<float>(),
                   inv_psi.data_ptr<float>(), cur_stream());
}

// Native pinned-ring prefetcher (residency=stream).  Holds references to the host dataset and
// staging tensors so their storage outlives the worker threads.
class HostPrefetcher {
 public:
  HostPrefetcher(std::vector<at::Tensor> host, std::vector<at::Tensor> staging, int64_t B, int64_t R,
                 int64_t nthreads)
      : host_(std::move(host)), staging_(std::move(staging)) {
    TORCH_CHECK(host_.size() == staging_.size() && !host_.empty(), "prefetch: host/staging tensor lists differ");
    std::vector<const void*> hp;
    std::vector<void*> sp;
    std::vector<long> rb;
    for (size_t t = 0; t < host_.size(); ++t) {
      auto& h = host_[t];
      auto& s = staging_[t];
      TORCH_CHECK(!h.is_cuda() && h.is_contiguous(), "prefetch: host tensors must be contiguous CPU tensors");
      TORCH_CHECK(!s.is_cuda() && s.is_contiguous() && s.dtype() == h.dtype(), "prefetch: bad staging tensor");
      const long row = h.dim() > 1 ? (long)(h.numel() / h.size(0)) * (long)h.element_size() : (long)h.element_size();
      TORCH_CHECK((long)s.numel() * (long)s.element_size() >= (long)(R * B) * row, "prefetch: staging too small");
      hp.push_back(h.data_ptr());
      sp.push_back(s.data_ptr());
      rb.push_back(row);
      rows_ = h.size(0);
    }
    h_ = mta_prefetch_create((int)host_.size(), hp.data(), rb.data(), sp.data(), (int)B, (int)R, (int)nthreads);
  }
  ~HostPrefetcher() { close(); }
  void start(at::Tensor idx, int64_t n_batches) {
    TORCH_CHECK(!idx.is_cuda() && idx.dtype() == at::kLong && idx.is_contiguous(), "prefetch: idx must be int64 CPU");
    if (idx.numel()) {
      TORCH_CHECK(idx.min().item<int64_t>() >= 0 && idx.max().item<int64_t>() < rows_, "prefetch: index out of range");
    }
    idx_ = idx;
    mta_prefetch_start(h_, idx.data_ptr<int64_t>(), (long)idx.numel(), (long)n_batches);
  }
  int64_t wait(int64_t b, int64_t timeout_ms) {
    py::gil_scoped_release nogil;
    return mta_prefetch_wait(h_, (long)b, (long)timeout_ms);
  }
  bool ready(int64_t b) { return mta_prefetch_ready(h_, (long)b) != 0; }
  void release(int64_t b) { mta_prefetch_release(h_, (long)b); }
  void stop() {
    py::gil_scoped_release nogil;
    if (h_) mta_prefetch_stop(h_);
  }
  void close() {
    if (h_) {
      py::gil_scoped_release nogil;
      mta_prefetch_destroy(h_);
      h_ = nullptr;
    }
  }

 private:
  std::vector<at::Tensor> host_, staging_;
  at::Tensor idx_;
  int64_t rows_ = 0;
  void* h_ = nullptr;
};

// Node census of a captured HIP graph (torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()): the type of every
// node, child graphs walked recursively.  The trainer's step graphs must hold kernel nodes only (a captured memset
// node was the root of the r3 multi-process NaN, profiles/r4_nan_root_cause.txt); tests assert it.
static void graph_node_types_rec(hipGraph_t g, std::vector<int64_t>& out, int depth) {
  size_t n = 0;
  TORCH_CHECK(hipGraphGetNodes(g, nullptr, &n) == hipSuccess, "hipGraphGetNodes (count) failed");
  std::vector<hipGraphNode_t> nodes(n);
  if (n) TORCH_CHECK(hipGraphGetNodes(g, nodes.data(), &n) == hipSuccess, "hipGraphGetNodes failed");
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    TORCH_CHECK(hipGraphNodeGetType(nodes[i], &t) == hipSuccess, "hipGraphNodeGetType failed");
    if (t == hipGraphNodeTypeGraph && depth < 8) {
      hipGraph_t child;
      TORCH_CHECK(hipGraphChildGraphNodeGetGraph(nodes[i], &child) == hipSuccess, "child graph lookup failed");
      graph_node_types_rec(child, out, depth + 1);
    } else {
      out.push_back((int64_t)t);
    }
  }
}

static std::vector<int64_t> graph_node_types(int64_t graph) {
  TORCH_CHECK(graph != 0, "graph_node_types: null graph (capture with keep_graph=True)");
  std::vector<int64_t> out;
  graph_node_types_rec(reinterpret_cast<hipGraph_t>(graph), out, 0);
  return out;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  py::class_<HostPrefetcher>(m, "HostPrefetcher")
      .def(py::init<std::vector<at::Tensor>, std::vector<at::Tensor>, int64_t, int64_t, int64_t>())
      .def("start", &HostPrefetcher::start)
      .def("wait", &HostPrefetcher::wait, py::arg("batch"), py::arg("timeout_ms") = -1)
      .def("ready", &HostPrefetcher::ready)
      .def("release", &HostPrefetcher::release)
      .def("stop", &HostPrefetcher::stop)
      .def("close", &HostPrefetcher::close);
  m.doc() = "masters_thesis_amd CDNA4 (gfx950) HIP kernels";
  m.def("dgp", &dgp);
  m.def("graph_node_types", &graph_node_types);
  m.attr("GRAPH_NODE_KERNEL") = (int64_t)hipGraphNodeTypeKernel;
  m.attr("GRAPH_NODE_MEMCPY") = (int64_t)hipGraphNodeTypeMemcpy;
  m.attr("GRAPH_NODE_MEMSET") = (int64_t)hipGraphNodeTypeMemset;
  m.def("ols_features", &ols_features);
  m.def("lstm_stack_fwd", &lstm_stack_fwd);
  m.def("lstm_stack_fwd_gather", &lstm_stack_fwd_gather);
  m.def("lstm_stack_bwd", &lstm_stack_bwd);
  m.def("lstm_stack_flag_words", &lstm_stack_flag_words);
  m.def("lstm_stack_epoch_shift", [](int64_t T) { return (int64_t)mta_lstm_stack_epoch_shift((int)T); });
  m.def("gemm_bf16", &gemm_bf16);
  m.def("gemm_flush", []() { mta_gemm_flush(); });
  m.def("gemm_f32x", &gemm_f32x, py::arg("prec"), py::arg("A"), py::arg("a_km"), py::arg("lda"), py::arg("B"),
        py::arg("b_kn"), py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("n_store"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("flags"), py::arg("bias"), py::arg("pre"), py::arg("mask") = py::none(),
        py::arg("resid") = py::none(), py::arg("seed") = py::none(), py::arg("drop_p") = 0.0);
  m.def("attention_f32", &attention_f32);
  m.def("colsum_f32", &colsum_f32);
  m.def("seeds_advance", [](at::Tensor seeds) {
    TORCH_CHECK(seeds.is_cuda() && seeds.scalar_type() == at::kLong && seeds.numel() <= 64, "seeds: int64[<= 64] GPU");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(seeds.device());
    mta_seeds_advance(reinterpret_cast<uint64_t*>(seeds.data_ptr<int64_t>()), (int)seeds.numel(), cur_stream());
  });
  // contiguous tensor <- 0 by a zero-fill KERNEL on the current stream.  A captured hipMemsetAsync (memset graph
  // node) was not ordered against the neighbouring kernel nodes on replay when several processes shared the GPU
  // (4-rank graphed transformer NaN, profiles/r4_nan_root_cause.txt): step graphs hold kernel nodes only
  // (tests/test_gpu_graphs.py)
  m.def("zero_", [](at::Tensor t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero_: contiguous GPU tensor");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
    mta_zero_bytes(t.data_ptr(), (long)(t.numel() * t.element_size()), cur_stream());
  });
  m.def("tr_ffn_fwd", &tr_ffn_fwd);
  m.def("frag_pack", &frag_pack, py::arg("src"), py::arg("dst"), py::arg("transposed"),
        py::arg("cast_src") = std::vector<at::Tensor>{}, py::arg("cast_dst") = std::vector<at::Tensor>{},
        py::arg("seeds") = py::none());
  m.def("tr_ffn_bwd", &tr_ffn_bwd);
  m.def("transpose_bf16", &transpose_bf16);
  m.def("tr_attn_fwd", &tr_attn_fwd, py::arg("nseq"), py::arg("T"), py::arg("heads"), py::arg("eps"),
        py::arg("rope_base"), py::arg("x"), py::arg("wqkv"), py::arg("wo"), py::arg("g1"), py::arg("bqkv"),
        py::arg("bo"), py::arg("xn"), py::arg("r1"), py::arg("qkv"), py::arg("o"), py::arg("lse"), py::arg("x1"),
        py::arg("in") = py::none(), py::arg("we") = py::none(), py::arg("be") = py::none());
  m.def("gemm_set_big", [](int64_t on) { mta_gemm_set_big((int)on); });
  m.def("norm_defer", []() { mta_norm_defer(); });
  m.def("gemm_group_flush", []() { mta_gemm_group_flush(); });
  m.def("gemm_group_discard", []() { mta_gemm_group_discard(); });
  m.def("norm_discard", []() { mta_norm_discard(); });
  m.def("norm_flush", []() { mta_norm_flush(); });
  m.def("cast_pad", &cast_pad, py::arg("src"), py::arg("dst"), py::arg("seeds") = py::none());
  m.def("pair_colsum", &pair_colsum);
  m.def("norm", &norm, py::arg("bwd"), py::arg("x"), py::arg("ldx"), py::arg("M"), py::arg("D"), py::arg("rms"),
        py::arg("eps"), py::arg("gamma"), py::arg("beta"), py::arg("y_bf16"), py::arg("y_f32"), py::arg("mean"),
        py::arg("rstd"), py::arg("seed"), py::arg("drop_p"), py::arg("dy"), py::arg("dres"), py::arg("pre"),
        py::arg("dx_bf16"), py::arg("dx_f32"), py::arg("dgamma"), py::arg("dbeta"), py::arg("gelu_x") = false,
        py::arg("hw_a") = py::none(), py::arg("hb_a") = py::none(), py::arg("hw_b") = py::none(),
        py::arg("hb_b") = py::none(), py::arg("ab") = py::none(), py::arg("ab_rows") = 0,
        py::arg("g_wa") = py::none(), py::arg("g_wb") = py::none());
  m.def("tr_attn_dx", &tr_attn_dx);
  m.def("attention", &attention, py::arg("bwd"), py::arg("qkv"), py::arg("out"), py::arg("lse"), py::arg("dout"),
        py::arg("dqkv"), py::arg("nseq"), py::arg("T"), py::arg("D"), py::arg("heads"), py::arg("rope_base"),
        py::arg("dx1") = py::none(), py::arg("wot") = py::none());
  m.def("lstm_fwd_layer", &lstm_fwd_layer);
  m.def("lstm_bwd_layer", &lstm_bwd_layer);
  m.def("lstm_wgrad", &lstm_wgrad);
  m.def("lstm_prep", &lstm_prep);
  m.def("gemm_f32", &gemm_f32);
  m.def("gather_batch", &gather_batch);
  m.def("decoder_losses", &decoder_losses);
  m.def("heads_losses", &heads_losses);
  m.def("heads_losses_bwd", &heads_losses_bwd);
  m.def("optim_num_partials", &optim_num_partials);
  m.def("grad_sqnorm", &grad_sqnorm);
  m.def("adam", &adam);
  m.def("xgmi_buffer_bytes", &xgmi_buffer_bytes);
  m.def("xgmi_alloc", &xgmi_alloc);
  m.def("xgmi_free", &xgmi_free);
  m.def("xgmi_ipc_handle", &xgmi_ipc_handle);
  m.def("xgmi_ipc_open", &xgmi_ipc_open);
  m.def("xgmi_ipc_close", &xgmi_ipc_close);
  m.def("xgmi_allreduce", &xgmi_allreduce);
  m.def("xgmi_ctl_words", []() { return (int64_t)mta_xgmi_ctl_words(); });
  m.def("set_heads_deterministic", [](bool on) { mta_set_heads_deterministic(on ? 1 : 0); });
  m.def("xgmi_max_channels", []() { return (int64_t)mta_xgmi_max_channels(); });
  m.def("xgmi_timeout_word", []() { return (int64_t)mta_xgmi_timeout_word(); });
  m.def("xgmi_max_blocks", []() { return (int64_t)mta_xgmi_max_blocks(); });
  m.def("lstm_wgrad_part_floats", [](int64_t fused, int64_t T, int64_t H, int64_t F) {
    return (int64_t)mta_lstm_wgrad_part_floats((int)fused, (int)T, (int)H, (int)F);
  });
  m.def("heads_losses_train", &heads_losses_train);
  m.def("adam_fused_partials", &adam_fused_partials);
  m.def("adam_fused", &adam_fused);
  m.def("gemm_grad_producer", &gemm_grad_producer);
  m.def("gemm_norm_parts", []() { return (int64_t)mta_gemm_norm_parts(); });
  m.def("scale_", &scale_);
  m.attr("ARCH") = "gfx950";
}
