// PyTorch bindings for the masters_thesis_amd HIP kernels (masters_thesis_amd._C).
// Kernels are plain HIP launchers (extern "C", raw pointers + hipStream_t); this file only
// validates tensors and forwards the current PyTorch HIP stream, so every op is stream-ordered
// with PyTorch and capturable into a HIP graph.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime.h>

extern "C" {
int mta_lstm_fwd_layer(int H, int prec, const float* x, const float* w_ih, const float* b_ih, const float* b_hh,
                       int fin, const float* gx, float* gates, const float* w_hh, float* hseq, float* cseq, int N,
                       int T, hipStream_t st);
int mta_lstm_bwd_layer(int H, int prec, float* gates, const float* cseq, const float* w_hh, const float* dH,
                       const float* dh_last, int N, int T, hipStream_t st);
void mta_decoder_losses(const float* ab, const float* y, const float* factor, const float* inv_psi, int N, int n,
                        int C, int windows, int kwin, int factor_stride, int want_nll, float* out, float* gmse,
                        float* gnll, hipStream_t st);
void mta_decoder_losses_bwd(const float* gout, const float* gmse, const float* gnll, float* dab, int N, int has_nll,
                            hipStream_t st);
int mta_optim_num_partials(long n);
void mta_grad_sqnorm(const float* g, long n, float scale, float* partials, float* step, hipStream_t st);
void mta_adam(float* p, float* g, float* m, float* v, long n, const float* partials, const float* lr,
              const float* step, float beta1, float beta2, float eps, float wd, float max_norm, float scale, int adamw,
              float* norm_out, hipStream_t st);
void mta_scale(float* x, long n, float s, hipStream_t st);
}

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define MTA_CHECK_F32(t)                                                                            \
  TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor");                                           \
  TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32");                              \
  TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

const float* opt_ptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  MTA_CHECK_F32(*t);
  return t->data_ptr<float>();
}

void lstm_fwd_layer(int64_t H, int64_t prec, const c10::optional<at::Tensor>& x, const c10::optional<at::Tensor>& w_ih,
                    const c10::optional<at::Tensor>& b_ih, const c10::optional<at::Tensor>& b_hh,
                    const c10::optional<at::Tensor>& gx, at::Tensor gates, at::Tensor w_hh, at::Tensor hseq,
                    at::Tensor cseq, int64_t N, int64_t T) {
  MTA_CHECK_F32(gates);
  MTA_CHECK_F32(w_hh);
  MTA_CHECK_F32(hseq);
  MTA_CHECK_F32(cseq);
  TORCH_CHECK(gates.numel() == T * N * 4 * H, "gates must be (T, N, 4H)");
  TORCH_CHECK(hseq.numel() == T * N * H && cseq.numel() == T * N * H, "hseq/cseq must be (T, N, H)");
  TORCH_CHECK(w_hh.numel() == 4 * H * H, "w_hh must be (4H, H)");
  int fin = 0;
  if (x.has_value() && x->defined()) {
    TORCH_CHECK(x->dim() == 3 && x->size(0) == N && x->size(1) == T, "x must be (N, T, F)");
    fin = (int)x->size(2);
    TORCH_CHECK(fin >= 1 && fin <= 5, "fused input projection supports 1 <= F <= 5");
    TORCH_CHECK(w_ih.has_value() && w_ih->numel() == 4 * H * fin, "w_ih must be (4H, F)");
    TORCH_CHECK(b_ih.has_value() && b_hh.has_value(), "fused input projection needs b_ih and b_hh");
  } else {
    TORCH_CHECK(gx.has_value() && gx->numel() == T * N * 4 * H, "gx must be (T, N, 4H)");
  }
  c10::hip::HIPGuard guard(gates.device());
  int rc = mta_lstm_fwd_layer((int)H, (int)prec, opt_ptr(x), opt_ptr(w_ih), opt_ptr(b_ih), opt_ptr(b_hh), fin,
                              opt_ptr(gx), gates.data_ptr<float>(), w_hh.data_ptr<float>(), hseq.data_ptr<float>(),
                              cseq.data_ptr<float>(), (int)N, (int)T, cur_stream());
  TORCH_CHECK(rc == 0, "lstm_fwd_layer: unsupported hidden size ", H, " (supported: 32, 64, 128)");
}

void lstm_bwd_layer(int64_t H, int64_t prec, at::Tensor gates, at::Tensor cseq, at::Tensor w_hh,
                    const c10::optional<at::Tensor>& dH, const c10::optional<at::Tensor>& dh_last, int64_t N,
                    int64_t T) {
  MTA_CHECK_F32(gates);
  MTA_CHECK_F32(cseq);
  MTA_CHECK_F32(w_hh);
  TORCH_CHECK(gates.numel() == T * N * 4 * H && cseq.numel() == T * N * H, "bad gates/cseq shape");
  if (dH.has_value() && dH->defined()) TORCH_CHECK(dH->numel() == T * N * H, "dH must be (T, N, H)");
  if (dh_last.has_value() && dh_last->defined()) TORCH_CHECK(dh_last->numel() == N * H, "dh_last must be (N, H)");
  c10::hip::HIPGuard guard(gates.device());
  int rc = mta_lstm_bwd_layer((int)H, (int)prec, gates.data_ptr<float>(), cseq.data_ptr<float>(),
                              w_hh.data_ptr<float>(), opt_ptr(dH), opt_ptr(dh_last), (int)N, (int)T, cur_stream());
  TORCH_CHECK(rc == 0, "lstm_bwd_layer: unsupported hidden size ", H);
}

void decoder_losses(at::Tensor ab, at::Tensor y, at::Tensor factor, at::Tensor inv_psi, int64_t windows,
                    int64_t kwin, int64_t factor_stride, bool want_nll, at::Tensor out, at::Tensor gmse,
                    at::Tensor gnll) {
  MTA_CHECK_F32(ab);
  MTA_CHECK_F32(y);
  MTA_CHECK_F32(factor);
  MTA_CHECK_F32(inv_psi);
  MTA_CHECK_F32(out);
  MTA_CHECK_F32(gmse);
  MTA_CHECK_F32(gnll);
  const int64_t N = ab.size(0);
  TORCH_CHECK(ab.dim() == 2 && ab.size(1) == 2, "ab must be (N, 2)");
  TORCH_CHECK(y.dim() == 3 && y.size(0) == N && y.size(2) >= 2, "y must be (N, n, C>=2)");
  TORCH_CHECK(inv_psi.numel() == N, "inv_psi must be (N,)");
  TORCH_CHECK(windows * kwin == N, "windows * kwin must equal N");
  TORCH_CHECK(factor.numel() >= 2 + (windows - 1) * factor_stride, "factor too small");
  TORCH_CHECK(out.numel() >= 4 && gmse.numel() == 2 * N && gnll.numel() == 2 * N, "bad output shapes");
  c10::hip::HIPGuard guard(ab.device());
  mta_decoder_losses(ab.data_ptr<float>(), y.data_ptr<float>(), factor.data_ptr<float>(), inv_psi.data_ptr<float>(),
                     (int)N, (int)y.size(1), (int)y.size(2), (int)windows, (int)kwin, (int)factor_stride,
                     want_nll ? 1 : 0, out.data_ptr<float>(), gmse.data_ptr<float>(), gnll.data_ptr<float>(),
                     cur_stream());
}

void decoder_losses_bwd(at::Tensor gout, at::Tensor gmse, at::Tensor gnll, at::Tensor dab, bool has_nll) {
  MTA_CHECK_F32(gout);
  MTA_CHECK_F32(gmse);
  MTA_CHECK_F32(gnll);
  MTA_CHECK_F32(dab);
  TORCH_CHECK(gout.numel() >= 2, "gout must hold [g_mse, g_nll]");
  c10::hip::HIPGuard guard(dab.device());
  mta_decoder_losses_bwd(gout.data_ptr<float>(), gmse.data_ptr<float>(), gnll.data_ptr<float>(),
                         dab.data_ptr<float>(), (int)(dab.numel() / 2), has_nll ? 1 : 0, cur_stream());
}

int64_t optim_num_partials(int64_t n) { return mta_optim_num_partials((long)n); }

void grad_sqnorm(at::Tensor g, double scale, at::Tensor partials, const c10::optional<at::Tensor>& step) {
  MTA_CHECK_F32(g);
  MTA_CHECK_F32(partials);
  TORCH_CHECK(g.numel() % 4 == 0, "flat buffers must be padded to a multiple of 4");
  TORCH_CHECK(partials.numel() >= mta_optim_num_partials((long)g.numel()), "partials too small");
  c10::hip::HIPGuard guard(g.device());
  float* stp = nullptr;
  if (step.has_value() && step->defined()) {
    MTA_CHECK_F32(*step);
    stp = step->data_ptr<float>();
  }
  mta_grad_sqnorm(g.data_ptr<float>(), (long)g.numel(), (float)scale, partials.data_ptr<float>(), stp, cur_stream());
}

void adam(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor partials, at::Tensor lr, at::Tensor step,
          double beta1, double beta2, double eps, double wd, double max_norm, double scale, bool adamw,
          const c10::optional<at::Tensor>& norm_out) {
  MTA_CHECK_F32(p);
  MTA_CHECK_F32(g);
  MTA_CHECK_F32(m);
  MTA_CHECK_F32(v);
  MTA_CHECK_F32(partials);
  MTA_CHECK_F32(lr);
  MTA_CHECK_F32(step);
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && n % 4 == 0, "flat buffer size mismatch");
  c10::hip::HIPGuard guard(p.device());
  float* no = nullptr;
  if (norm_out.has_value() && norm_out->defined()) {
    MTA_CHECK_F32(*norm_out);
    no = norm_out->data_ptr<float>();
  }
  mta_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), (long)n,
           partials.data_ptr<float>(), lr.data_ptr<float>(), step.data_ptr<float>(), (float)beta1, (float)beta2,
           (float)eps, (float)wd, (float)max_norm, (float)scale, adamw ? 1 : 0, no, cur_stream());
}

void scale_(at::Tensor x, double s) {
  MTA_CHECK_F32(x);
  TORCH_CHECK(x.numel() % 4 == 0, "flat buffers must be padded to a multiple of 4");
  c10::hip::HIPGuard guard(x.device());
  mta_scale(x.data_ptr<float>(), (long)x.numel(), (float)s, cur_stream());
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "masters_thesis_amd CDNA4 (gfx950) HIP kernels";
  m.def("lstm_fwd_layer", &lstm_fwd_layer);
  m.def("lstm_bwd_layer", &lstm_bwd_layer);
  m.def("decoder_losses", &decoder_losses);
  m.def("decoder_losses_bwd", &decoder_losses_bwd);
  m.def("optim_num_partials", &optim_num_partials);
  m.def("grad_sqnorm", &grad_sqnorm);
  m.def("adam", &adam);
  m.def("scale_", &scale_);
  m.attr("ARCH") = "gfx950";
}
