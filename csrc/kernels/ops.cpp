// torch.library registration of the mihvd HIP kernels: torch.ops.mihvd.<name>.
// All ops launch on the current HIP stream and allocate nothing, so they can be captured into a
// HIP graph by torch.cuda.graph.
#include <ATen/ATen.h>
#include <torch/library.h>

namespace mihvd {
void conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1);
void conv2_fwd(const at::Tensor& a1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2);
void conv12_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                const at::Tensor& w1bf, const at::Tensor& b1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a1,
                at::Tensor& idx1, at::Tensor& a2, at::Tensor& idx2, int64_t coll);
void fc1_fwd(const at::Tensor& a2, const at::Tensor& w3bf, at::Tensor& zpart);
void fc1_bwd(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog,
             const at::Tensor& w3bf, at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, at::Tensor& g2,
             int64_t roles, int64_t coll, const c10::optional<at::Tensor>& a2T,
             const c10::optional<at::Tensor>& dzT);
void head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                  const at::Tensor& labels, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                  int64_t seed, double rate, at::Tensor& h, at::Tensor& dz, at::Tensor& dlog, at::Tensor& stats,
                  int64_t coll, double dz_scale, const c10::optional<at::Tensor>& stats_acc,
                  const c10::optional<at::Tensor>& loss_scale);
void fc1_wgrad(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog, at::Tensor& gW3,
               at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, int64_t roles, const c10::optional<at::Tensor>& dz_w3,
               const c10::optional<at::Tensor>& a2_w3, int64_t jt_lo, int64_t jt_hi, int64_t coll);
void fc1_wgrad_adam(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog,
                    at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, int64_t roles,
                    const c10::optional<at::Tensor>& dz_w3, const c10::optional<at::Tensor>& a2_w3, at::Tensor& p3,
                    at::Tensor& m3, at::Tensor& v3, at::Tensor& shadow3, const at::Tensor& state, double lr, double b1,
                    double b2, double eps, double grad_scale, int64_t rule, bool write_grad, int64_t jt_lo,
                    int64_t jt_hi, int64_t coll);
void fc1_dgrad(const at::Tensor& dz, const at::Tensor& w3bf, const at::Tensor& a2, at::Tensor& g2);
int64_t conv2_wgrad_groups(int64_t B);
void conv2_bwd(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
               const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, const c10::optional<at::Tensor>& g1,
               int64_t coll);
void conv2_wgrad_reduce(const at::Tensor& slab, const at::Tensor& cpart, int64_t B, at::Tensor& gW2, at::Tensor& gW1,
                        at::Tensor& gb1, at::Tensor& gb2);
void conv2_bwd_adam(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                    const at::Tensor& x, const c10::optional<at::Tensor>& rows, at::Tensor& state, const at::Tensor& idx1,
                    at::Tensor& slab, at::Tensor& cpart, at::Tensor& p3, const at::Tensor& g3, at::Tensor& m3,
                    at::Tensor& v3, at::Tensor& shadow3, double lr, double b1, double b2, double eps, double grad_scale,
                    int64_t rule);
void conv2_bwd_w3adam(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                      const at::Tensor& x, const c10::optional<at::Tensor>& rows, at::Tensor& state,
                      const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, const at::Tensor& dzT,
                      const at::Tensor& a2T, at::Tensor& p3, at::Tensor& m3, at::Tensor& v3, at::Tensor& shadow3,
                      const c10::optional<at::Tensor>& gW3, double lr, double b1, double b2, double eps,
                      double grad_scale, int64_t rule);
void conv2_wgrad_reduce_adam(const at::Tensor& slab, const at::Tensor& cpart, int64_t B, at::Tensor& gW2,
                             at::Tensor& gW1, at::Tensor& gb1, at::Tensor& gb2, const at::Tensor& grads, at::Tensor& p,
                             at::Tensor& m, at::Tensor& v, at::Tensor& shadow, at::Tensor& state, int64_t fc_lo,
                             int64_t w3_lo, double lr, double b1, double b2, double eps, double grad_scale,
                             int64_t rule);
void conv2_bwd_adam_fold(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                         const at::Tensor& x, const c10::optional<at::Tensor>& rows, at::Tensor& state,
                         const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, at::Tensor& gW2, at::Tensor& gW1,
                         at::Tensor& gb1, at::Tensor& gb2, const at::Tensor& grads, at::Tensor& p, at::Tensor& m,
                         at::Tensor& v, at::Tensor& shadow, at::Tensor& sync, int64_t fc_lo, int64_t w3_lo, double lr,
                         double b1, double b2, double eps, double grad_scale, int64_t rule);
void adam_step(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, const c10::optional<at::Tensor>& shadow,
               const c10::optional<at::Tensor>& state, int64_t host_step, double lr, double b1, double b2, double eps,
               double grad_scale, int64_t rule, int64_t bump, const c10::optional<at::Tensor>& loss_scale,
               int64_t max_blocks);
void scale_cast_bf16(const at::Tensor& src, at::Tensor& dst, double scale);
void bf16_to_f32(const at::Tensor& src, at::Tensor& dst, double scale);
void scale_cast_f16(const at::Tensor& src, at::Tensor& dst, double scale);
void f16_to_f32(const at::Tensor& src, at::Tensor& dst, double scale);
void segment_dots(const at::Tensor& a, const at::Tensor& b, const at::Tensor& offs_dev, int64_t max_seg_len,
                  at::Tensor& out);
void adasum_combine(const at::Tensor& a, const at::Tensor& b, const at::Tensor& offs_dev, int64_t max_seg_len,
                    const at::Tensor& dots, at::Tensor& out);
void grad_check_(at::TensorList grads, at::Tensor& ls, bool unscale);
void update_scale_(at::Tensor& ls, at::Tensor& tracker, double growth, double backoff, int64_t interval,
                   double min_scale, const c10::optional<at::Tensor>& state);
void gather_cols_bf16(const at::Tensor& src, int64_t col0, at::Tensor& dst);
void multi_tensor_adam(std::vector<at::Tensor> p, std::vector<at::Tensor> g, std::vector<at::Tensor> m,
                       std::vector<at::Tensor> v, const c10::optional<at::Tensor>& step, int64_t host_step, double lr,
                       double b1, double b2, double eps, double weight_decay, bool decoupled, int64_t rule,
                       double grad_scale);
void multi_tensor_sgd(std::vector<at::Tensor> p, std::vector<at::Tensor> g, std::vector<at::Tensor> bufs, double lr,
                      double momentum, double dampening, double weight_decay, bool nesterov, bool first,
                      double grad_scale);
void bump_step_(at::Tensor& step);
void f32_conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                   const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1,
                   const c10::optional<at::Tensor>& w2, const c10::optional<at::Tensor>& w2frag, int64_t coll,
                   const c10::optional<at::Tensor>& xpre);
void f32_prime_batch(const at::Tensor& x, const at::Tensor& labels, const at::Tensor& rows, const at::Tensor& state,
                     at::Tensor& xpre, at::Tensor& ypre);
void f32_conv2_fwd(const at::Tensor& a1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2,
                   const c10::optional<at::Tensor>& w2frag, int64_t products);
void f32_fc1_fwd(const at::Tensor& a2, const at::Tensor& w3, at::Tensor& zpart, int64_t products);
void f32_head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                      const at::Tensor& labels, const c10::optional<at::Tensor>& rows,
                      const c10::optional<at::Tensor>& state, int64_t seed, double rate, at::Tensor& h, at::Tensor& dz,
                      at::Tensor& dlog, at::Tensor& stats, const c10::optional<at::Tensor>& stats_acc,
                      const c10::optional<at::Tensor>& ypre);
void f32_fc1_bwd(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& h,
                 const at::Tensor& dlog, at::Tensor& w3, at::Tensor& dY2, at::Tensor& db2p, at::Tensor& gW3,
                 at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, const c10::optional<at::Tensor>& m3,
                 const c10::optional<at::Tensor>& v3, const c10::optional<at::Tensor>& state, double lr, double beta1,
                 double beta2, double eps, double grad_scale, int64_t rule, bool store_w3,
                 const c10::optional<at::Tensor>& px, const c10::optional<at::Tensor>& plabels,
                 const c10::optional<at::Tensor>& prows, const c10::optional<at::Tensor>& pstate,
                 const c10::optional<at::Tensor>& xpre, const c10::optional<at::Tensor>& ypre);
void f32_conv2_bwd(const at::Tensor& dY2, const at::Tensor& w2, const at::Tensor& a1, const at::Tensor& idx1,
                   const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                   at::Tensor& cpart, at::Tensor& slab, const c10::optional<at::Tensor>& w2frag, int64_t products);
void f32_factor_rows(const at::Tensor& a2c, const at::Tensor& dz, const c10::optional<at::Tensor>& out,
                     const c10::optional<at::Tensor>& p, const c10::optional<at::Tensor>& m,
                     const c10::optional<at::Tensor>& v, const c10::optional<at::Tensor>& state, double lr,
                     double beta1, double beta2, double eps, double grad_scale, int64_t rule);
void f32_factor_full(const at::Tensor& a2, const at::Tensor& dz, int64_t B, const c10::optional<at::Tensor>& out,
                     at::Tensor& p, at::Tensor& m, at::Tensor& v, const at::Tensor& state, double lr, double beta1,
                     double beta2, double eps, double grad_scale, int64_t rule);
void f32_conv_reduce(const at::Tensor& slab, const at::Tensor& cpart, const at::Tensor& db2p, at::Tensor& gW2,
                     at::Tensor& gW1, at::Tensor& gb1, at::Tensor& gb2, const c10::optional<at::Tensor>& params,
                     const c10::optional<at::Tensor>& grads, const c10::optional<at::Tensor>& m,
                     const c10::optional<at::Tensor>& v, const c10::optional<at::Tensor>& state, int64_t o_w1,
                     int64_t o_b1, int64_t o_w2, int64_t o_b2, int64_t fc_lo, int64_t fc_hi, double lr, double b1,
                     double b2, double eps, double grad_scale, int64_t rule);
int64_t f32_db2_rows(int64_t B);
at::Tensor f32_stamps_enable(int64_t n_blocks, int64_t kernel);
int64_t f32_wgrad_groups(int64_t B, int64_t products);
int64_t f32_dgrad_blocks(int64_t B, int64_t products);
int64_t conv_barrier_error(bool reset);
}  // namespace mihvd

// The fp16-operand build of conv_fwd.hip / conv_bwd.hip / fc.hip (common.h, -DMIHVD_F16).
namespace mihvd {
namespace f16 {
void conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1);
void conv2_fwd(const at::Tensor& a1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2);
void conv12_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                const at::Tensor& w1bf, const at::Tensor& b1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a1,
                at::Tensor& idx1, at::Tensor& a2, at::Tensor& idx2, int64_t coll);
void fc1_fwd(const at::Tensor& a2, const at::Tensor& w3bf, at::Tensor& zpart);
void fc1_bwd(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog,
             const at::Tensor& w3bf, at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, at::Tensor& g2,
             int64_t roles, int64_t coll, const c10::optional<at::Tensor>& a2T,
             const c10::optional<at::Tensor>& dzT);
void head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                  const at::Tensor& labels, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                  int64_t seed, double rate, at::Tensor& h, at::Tensor& dz, at::Tensor& dlog, at::Tensor& stats,
                  int64_t coll, double dz_scale, const c10::optional<at::Tensor>& stats_acc,
                  const c10::optional<at::Tensor>& loss_scale);
void conv2_bwd(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
               const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, const c10::optional<at::Tensor>& g1,
               int64_t coll);
}  // namespace f16
}  // namespace mihvd

namespace {

using at::Tensor;
using OptT = c10::optional<at::Tensor>;

void conv1_fwd_op(const Tensor& x, const OptT& rows, const OptT& state, const Tensor& w1, const Tensor& b1, Tensor a1,
                  Tensor idx1) {
  mihvd::conv1_fwd(x, rows, state, w1, b1, a1, idx1);
}
void conv2_fwd_op(const Tensor& a1, const Tensor& w2, const Tensor& b2, Tensor a2, Tensor idx2) {
  mihvd::conv2_fwd(a1, w2, b2, a2, idx2);
}
void conv12_fwd_op(const Tensor& x, const c10::optional<Tensor>& rows, const c10::optional<Tensor>& state,
                   const Tensor& w1, const Tensor& b1, const Tensor& w2, const Tensor& b2, Tensor a1, Tensor idx1,
                   Tensor a2, Tensor idx2, int64_t coll) {
  mihvd::conv12_fwd(x, rows, state, w1, b1, w2, b2, a1, idx1, a2, idx2, coll);
}
void fc1_bwd_op(const Tensor& dz, const Tensor& a2, const Tensor& h, const Tensor& dlog, const Tensor& w3, Tensor gW3,
               Tensor gb3, Tensor gW4, Tensor gb4, Tensor g2, int64_t roles, int64_t coll, const OptT& a2T,
               const OptT& dzT) {
  mihvd::fc1_bwd(dz, a2, h, dlog, w3, gW3, gb3, gW4, gb4, g2, roles, coll, a2T, dzT);
}
void fc1_fwd_op(const Tensor& a2, const Tensor& w3, Tensor zpart) { mihvd::fc1_fwd(a2, w3, zpart); }
void head_op(const Tensor& zpart, const Tensor& b3, const Tensor& w4, const Tensor& b4, const Tensor& labels,
             const OptT& rows, const OptT& state, int64_t seed, double rate, Tensor h, Tensor dz, Tensor dlog, Tensor stats,
             int64_t coll, double dz_scale, const OptT& stats_acc, const OptT& loss_scale) {
  mihvd::head_fwd_bwd(zpart, b3, w4, b4, labels, rows, state, seed, rate, h, dz, dlog, stats, coll, dz_scale, stats_acc,
                      loss_scale);
}
// fp16-operand ops (the Keras mixed_float16 policy): the bf16 ops' schemas, half tensors.
void conv1_fwd_f16_op(const Tensor& x, const OptT& rows, const OptT& state, const Tensor& w1, const Tensor& b1,
                      Tensor a1, Tensor idx1) {
  mihvd::f16::conv1_fwd(x, rows, state, w1, b1, a1, idx1);
}
void conv2_fwd_f16_op(const Tensor& a1, const Tensor& w2, const Tensor& b2, Tensor a2, Tensor idx2) {
  mihvd::f16::conv2_fwd(a1, w2, b2, a2, idx2);
}
void conv12_fwd_f16_op(const Tensor& x, const OptT& rows, const OptT& state, const Tensor& w1, const Tensor& b1,
                       const Tensor& w2, const Tensor& b2, Tensor a1, Tensor idx1, Tensor a2, Tensor idx2, int64_t coll) {
  mihvd::f16::conv12_fwd(x, rows, state, w1, b1, w2, b2, a1, idx1, a2, idx2, coll);
}
void fc1_fwd_f16_op(const Tensor& a2, const Tensor& w3, Tensor zpart) { mihvd::f16::fc1_fwd(a2, w3, zpart); }
void head_f16_op(const Tensor& zpart, const Tensor& b3, const Tensor& w4, const Tensor& b4, const Tensor& labels,
                 const OptT& rows, const OptT& state, int64_t seed, double rate, Tensor h, Tensor dz, Tensor dlog,
                 Tensor stats, int64_t coll, double dz_scale, const OptT& stats_acc, const OptT& loss_scale) {
  mihvd::f16::head_fwd_bwd(zpart, b3, w4, b4, labels, rows, state, seed, rate, h, dz, dlog, stats, coll, dz_scale,
                           stats_acc, loss_scale);
}
void fc1_bwd_f16_op(const Tensor& dz, const Tensor& a2, const Tensor& h, const Tensor& dlog, const Tensor& w3,
                    Tensor gW3, Tensor gb3, Tensor gW4, Tensor gb4, Tensor g2, int64_t roles, int64_t coll,
                    const OptT& a2T, const OptT& dzT) {
  mihvd::f16::fc1_bwd(dz, a2, h, dlog, w3, gW3, gb3, gW4, gb4, g2, roles, coll, a2T, dzT);
}
void conv2_bwd_f16_op(const Tensor& g2, const Tensor& idx2, const Tensor& a1, const Tensor& w2, const Tensor& x,
                      const OptT& rows, const OptT& state, const Tensor& idx1, Tensor slab, Tensor cpart,
                      const OptT& g1, int64_t coll) {
  mihvd::f16::conv2_bwd(g2, idx2, a1, w2, x, rows, state, idx1, slab, cpart, g1, coll);
}
void fc1_wgrad_op(const Tensor& dz, const Tensor& a2, const Tensor& h, const Tensor& dlog, Tensor gW3, Tensor gb3,
                  Tensor gW4, Tensor gb4, int64_t roles, const OptT& dz_w3, const OptT& a2_w3, int64_t jt_lo,
                  int64_t jt_hi, int64_t coll) {
  mihvd::fc1_wgrad(dz, a2, h, dlog, gW3, gb3, gW4, gb4, roles, dz_w3, a2_w3, jt_lo, jt_hi, coll);
}
void fc1_wgrad_adam_op(const Tensor& dz, const Tensor& a2, const Tensor& h, const Tensor& dlog, Tensor gW3, Tensor gb3,
                       Tensor gW4, Tensor gb4, int64_t roles, const OptT& dz_w3, const OptT& a2_w3, Tensor p3, Tensor m3,
                       Tensor v3, Tensor shadow3, const Tensor& state, double lr, double b1, double b2, double eps,
                       double grad_scale, int64_t rule, bool write_grad, int64_t jt_lo, int64_t jt_hi, int64_t coll) {
  mihvd::fc1_wgrad_adam(dz, a2, h, dlog, gW3, gb3, gW4, gb4, roles, dz_w3, a2_w3, p3, m3, v3, shadow3, state, lr, b1, b2,
                        eps, grad_scale, rule, write_grad, jt_lo, jt_hi, coll);
}
void fc1_dgrad_op(const Tensor& dz, const Tensor& w3, const Tensor& a2, Tensor g2) { mihvd::fc1_dgrad(dz, w3, a2, g2); }
void conv2_bwd_op(const Tensor& g2, const Tensor& idx2, const Tensor& a1, const Tensor& w2, const Tensor& x,
                  const OptT& rows, const OptT& state, const Tensor& idx1, Tensor slab, Tensor cpart, const OptT& g1,
                  int64_t coll) {
  mihvd::conv2_bwd(g2, idx2, a1, w2, x, rows, state, idx1, slab, cpart, g1, coll);
}
void conv2_wgrad_reduce_op(const Tensor& slab, const Tensor& cpart, int64_t B, Tensor gW2, Tensor gW1, Tensor gb1,
                           Tensor gb2) {
  mihvd::conv2_wgrad_reduce(slab, cpart, B, gW2, gW1, gb1, gb2);
}
void conv2_bwd_adam_op(const Tensor& g2, const Tensor& idx2, const Tensor& a1, const Tensor& w2, const Tensor& x,
                       const OptT& rows, Tensor state, const Tensor& idx1, Tensor slab, Tensor cpart, Tensor p3,
                       const Tensor& g3, Tensor m3, Tensor v3, Tensor shadow3, double lr, double b1, double b2,
                       double eps, double grad_scale, int64_t rule) {
  mihvd::conv2_bwd_adam(g2, idx2, a1, w2, x, rows, state, idx1, slab, cpart, p3, g3, m3, v3, shadow3, lr, b1, b2, eps,
                        grad_scale, rule);
}
void conv2_bwd_w3adam_op(const Tensor& g2, const Tensor& idx2, const Tensor& a1, const Tensor& w2, const Tensor& x,
                         const OptT& rows, Tensor state, const Tensor& idx1, Tensor slab, Tensor cpart, const Tensor& dzT,
                         const Tensor& a2T, Tensor p3, Tensor m3, Tensor v3, Tensor shadow3, const OptT& gW3, double lr,
                         double b1, double b2, double eps, double grad_scale, int64_t rule) {
  mihvd::conv2_bwd_w3adam(g2, idx2, a1, w2, x, rows, state, idx1, slab, cpart, dzT, a2T, p3, m3, v3, shadow3, gW3, lr, b1,
                          b2, eps, grad_scale, rule);
}
void conv2_wgrad_reduce_adam_op(const Tensor& slab, const Tensor& cpart, int64_t B, Tensor gW2, Tensor gW1, Tensor gb1,
                                Tensor gb2, const Tensor& grads, Tensor p, Tensor m, Tensor v, Tensor shadow,
                                Tensor state, int64_t fc_lo, int64_t w3_lo, double lr, double b1, double b2, double eps,
                                double grad_scale, int64_t rule) {
  mihvd::conv2_wgrad_reduce_adam(slab, cpart, B, gW2, gW1, gb1, gb2, grads, p, m, v, shadow, state, fc_lo, w3_lo, lr,
                                 b1, b2, eps, grad_scale, rule);
}
void conv2_bwd_adam_fold_op(const Tensor& g2, const Tensor& idx2, const Tensor& a1, const Tensor& w2, const Tensor& x,
                            const OptT& rows, Tensor state, const Tensor& idx1, Tensor slab, Tensor cpart, Tensor gW2,
                            Tensor gW1, Tensor gb1, Tensor gb2, const Tensor& grads, Tensor p, Tensor m, Tensor v,
                            Tensor shadow, Tensor sync, int64_t fc_lo, int64_t w3_lo, double lr, double b1, double b2,
                            double eps, double grad_scale, int64_t rule) {
  mihvd::conv2_bwd_adam_fold(g2, idx2, a1, w2, x, rows, state, idx1, slab, cpart, gW2, gW1, gb1, gb2, grads, p, m, v,
                             shadow, sync, fc_lo, w3_lo, lr, b1, b2, eps, grad_scale, rule);
}
void adam_op(Tensor p, const Tensor& g, Tensor m, Tensor v, const OptT& shadow, const OptT& state, int64_t host_step,
             double lr, double b1, double b2, double eps, double grad_scale, int64_t rule, int64_t bump,
             const OptT& loss_scale, int64_t max_blocks) {
  mihvd::adam_step(p, g, m, v, shadow, state, host_step, lr, b1, b2, eps, grad_scale, rule, bump, loss_scale,
                   max_blocks);
}
void scale_cast_op(const Tensor& src, Tensor dst, double scale) { mihvd::scale_cast_bf16(src, dst, scale); }
void bf16_to_f32_op(const Tensor& src, Tensor dst, double scale) { mihvd::bf16_to_f32(src, dst, scale); }
void scale_cast_f16_op(const Tensor& src, Tensor dst, double scale) { mihvd::scale_cast_f16(src, dst, scale); }
void f16_to_f32_op(const Tensor& src, Tensor dst, double scale) { mihvd::f16_to_f32(src, dst, scale); }
void segment_dots_op(const Tensor& a, const Tensor& b, const Tensor& offs, int64_t max_len, Tensor out) {
  mihvd::segment_dots(a, b, offs, max_len, out);
}
void adasum_combine_op(const Tensor& a, const Tensor& b, const Tensor& offs, int64_t max_len, const Tensor& dots,
                       Tensor out) {
  mihvd::adasum_combine(a, b, offs, max_len, dots, out);
}
void grad_check_op(at::TensorList grads, Tensor ls, bool unscale) { mihvd::grad_check_(grads, ls, unscale); }
void update_scale_op(Tensor ls, Tensor tracker, double growth, double backoff, int64_t interval, double min_scale,
                     const OptT& state) {
  mihvd::update_scale_(ls, tracker, growth, backoff, interval, min_scale, state);
}
void gather_cols_op(const Tensor& src, int64_t col0, Tensor dst) { mihvd::gather_cols_bf16(src, col0, dst); }
void mt_adam_op(at::TensorList p, at::TensorList g, at::TensorList m, at::TensorList v, const OptT& step,
                int64_t host_step, double lr, double b1, double b2, double eps, double wd, bool decoupled, int64_t rule,
                double grad_scale) {
  mihvd::multi_tensor_adam(p.vec(), g.vec(), m.vec(), v.vec(), step, host_step, lr, b1, b2, eps, wd, decoupled, rule,
                           grad_scale);
}
void mt_sgd_op(at::TensorList p, at::TensorList g, at::TensorList bufs, double lr, double momentum, double dampening,
               double wd, bool nesterov, bool first, double grad_scale) {
  mihvd::multi_tensor_sgd(p.vec(), g.vec(), bufs.vec(), lr, momentum, dampening, wd, nesterov, first, grad_scale);
}
void bump_step_op(Tensor step) { mihvd::bump_step_(step); }
void f32_conv1_op(const Tensor& x, const OptT& rows, const OptT& state, const Tensor& w1, const Tensor& b1, Tensor a1,
                  Tensor idx1, const OptT& w2, const OptT& w2frag, int64_t coll, const OptT& xpre) {
  mihvd::f32_conv1_fwd(x, rows, state, w1, b1, a1, idx1, w2, w2frag, coll, xpre);
}
void f32_prime_op(const Tensor& x, const Tensor& labels, const Tensor& rows, const Tensor& state, Tensor xpre,
                  Tensor ypre) {
  mihvd::f32_prime_batch(x, labels, rows, state, xpre, ypre);
}
void f32_conv2_op(const Tensor& a1, const Tensor& w2, const Tensor& b2, Tensor a2, Tensor idx2, const OptT& w2frag,
                  int64_t products) {
  mihvd::f32_conv2_fwd(a1, w2, b2, a2, idx2, w2frag, products);
}
void f32_fc1_fwd_op(const Tensor& a2, const Tensor& w3, Tensor zpart, int64_t products) {
  mihvd::f32_fc1_fwd(a2, w3, zpart, products);
}
void f32_head_op(const Tensor& zpart, const Tensor& b3, const Tensor& w4, const Tensor& b4, const Tensor& labels,
                 const OptT& rows, const OptT& state, int64_t seed, double rate, Tensor h, Tensor dz, Tensor dlog,
                 Tensor stats, const OptT& stats_acc, const OptT& ypre) {
  mihvd::f32_head_fwd_bwd(zpart, b3, w4, b4, labels, rows, state, seed, rate, h, dz, dlog, stats, stats_acc, ypre);
}
void f32_fc1_bwd_op(const Tensor& dz, const Tensor& a2, const Tensor& idx2, const Tensor& h, const Tensor& dlog,
                    Tensor w3, Tensor dY2, Tensor db2p, Tensor gW3, Tensor gb3, Tensor gW4, Tensor gb4, const OptT& m3,
                    const OptT& v3, const OptT& state, double lr, double beta1, double beta2, double eps,
                    double grad_scale, int64_t rule, bool store_w3, const OptT& px, const OptT& plabels,
                    const OptT& prows, const OptT& pstate, const OptT& xpre, const OptT& ypre) {
  mihvd::f32_fc1_bwd(dz, a2, idx2, h, dlog, w3, dY2, db2p, gW3, gb3, gW4, gb4, m3, v3, state, lr, beta1, beta2, eps,
                     grad_scale, rule, store_w3, px, plabels, prows, pstate, xpre, ypre);
}
void f32_conv2_bwd_op(const Tensor& dY2, const Tensor& w2, const Tensor& a1, const Tensor& idx1, const Tensor& x,
                      const OptT& rows, const OptT& state, Tensor cpart, Tensor slab, const OptT& w2frag,
                      int64_t products) {
  mihvd::f32_conv2_bwd(dY2, w2, a1, idx1, x, rows, state, cpart, slab, w2frag, products);
}
void f32_factor_rows_op(const Tensor& a2c, const Tensor& dz, const OptT& out, const OptT& p, const OptT& m,
                        const OptT& v, const OptT& state, double lr, double beta1, double beta2, double eps,
                        double grad_scale, int64_t rule) {
  mihvd::f32_factor_rows(a2c, dz, out, p, m, v, state, lr, beta1, beta2, eps, grad_scale, rule);
}
void f32_factor_full_op(const Tensor& a2, const Tensor& dz, int64_t B, const OptT& out, Tensor p, Tensor m, Tensor v,
                        const Tensor& state, double lr, double beta1, double beta2, double eps, double grad_scale,
                        int64_t rule) {
  mihvd::f32_factor_full(a2, dz, B, out, p, m, v, state, lr, beta1, beta2, eps, grad_scale, rule);
}
void f32_conv_reduce_op(const Tensor& slab, const Tensor& cpart, const Tensor& db2p, Tensor gW2, Tensor gW1, Tensor gb1,
                        Tensor gb2, const OptT& params, const OptT& grads, const OptT& m, const OptT& v,
                        const OptT& state, int64_t o_w1, int64_t o_b1, int64_t o_w2, int64_t o_b2, int64_t fc_lo,
                        int64_t fc_hi, double lr, double b1, double b2, double eps, double grad_scale, int64_t rule) {
  mihvd::f32_conv_reduce(slab, cpart, db2p, gW2, gW1, gb1, gb2, params, grads, m, v, state, o_w1, o_b1, o_w2, o_b2,
                         fc_lo, fc_hi, lr, b1, b2, eps, grad_scale, rule);
}
}  // namespace

TORCH_LIBRARY(mihvd, m) {
  m.def("conv1_fwd(Tensor x, Tensor? rows, Tensor? state, Tensor w1, Tensor b1, Tensor(a!) a1, Tensor(b!) idx1) -> ()");
  m.def("conv2_fwd(Tensor a1, Tensor w2bf, Tensor b2, Tensor(a!) a2, Tensor(b!) idx2) -> ()");
  m.def("conv12_fwd(Tensor x, Tensor? rows, Tensor? state, Tensor w1bf, Tensor b1, Tensor w2bf, Tensor b2, "
        "Tensor(a!) a1, Tensor(b!) idx1, Tensor(c!) a2, Tensor(d!) idx2, int coll=-1) -> ()");
  m.def("fc1_bwd(Tensor dz, Tensor a2, Tensor h, Tensor dlog, Tensor w3bf, Tensor(a!) gW3, Tensor(b!) gb3, "
        "Tensor(c!) gW4, Tensor(d!) gb4, Tensor(e!) g2, int roles=3, int coll=-1, Tensor(f!)? a2T=None, "
        "Tensor(g!)? dzT=None) -> ()");
  m.def("fc1_fwd(Tensor a2, Tensor w3bf, Tensor(a!) zpart) -> ()");
  m.def("head_fwd_bwd(Tensor zpart, Tensor b3, Tensor w4, Tensor b4, Tensor labels, Tensor? rows, Tensor(s!)? state, "
        "int seed, float rate, Tensor(a!) h, Tensor(b!) dz, Tensor(c!) dlog, Tensor(d!) stats, int coll=-1, "
        "float dz_scale=1., Tensor(e!)? stats_acc=None, Tensor? loss_scale=None) -> ()");
  m.def("conv1_fwd_f16(Tensor x, Tensor? rows, Tensor? state, Tensor w1, Tensor b1, Tensor(a!) a1, Tensor(b!) idx1) -> ()");
  m.def("conv2_fwd_f16(Tensor a1, Tensor w2h, Tensor b2, Tensor(a!) a2, Tensor(b!) idx2) -> ()");
  m.def("conv12_fwd_f16(Tensor x, Tensor? rows, Tensor? state, Tensor w1h, Tensor b1, Tensor w2h, Tensor b2, "
        "Tensor(a!) a1, Tensor(b!) idx1, Tensor(c!) a2, Tensor(d!) idx2, int coll=-1) -> ()");
  m.def("fc1_fwd_f16(Tensor a2, Tensor w3h, Tensor(a!) zpart) -> ()");
  m.def("head_fwd_bwd_f16(Tensor zpart, Tensor b3, Tensor w4, Tensor b4, Tensor labels, Tensor? rows, "
        "Tensor(s!)? state, int seed, float rate, Tensor(a!) h, Tensor(b!) dz, Tensor(c!) dlog, Tensor(d!) stats, "
        "int coll=-1, float dz_scale=1., Tensor(e!)? stats_acc=None, Tensor? loss_scale=None) -> ()");
  m.def("fc1_bwd_f16(Tensor dz, Tensor a2, Tensor h, Tensor dlog, Tensor w3h, Tensor(a!) gW3, Tensor(b!) gb3, "
        "Tensor(c!) gW4, Tensor(d!) gb4, Tensor(e!) g2, int roles=3, int coll=-1, Tensor(f!)? a2T=None, "
        "Tensor(g!)? dzT=None) -> ()");
  m.def("conv2_bwd_f16(Tensor g2, Tensor idx2, Tensor a1, Tensor w2h, Tensor x, Tensor? rows, Tensor? state, "
        "Tensor idx1, Tensor(a!) slab, Tensor(b!) cpart, Tensor(c!)? g1=None, int coll=-1) -> ()");
  m.def("fc1_wgrad(Tensor dz, Tensor a2, Tensor h, Tensor dlog, Tensor(a!) gW3, Tensor(b!) gb3, Tensor(c!) gW4, "
        "Tensor(d!) gb4, int roles=3, Tensor? dz_w3=None, Tensor? a2_w3=None, int jt_lo=0, int jt_hi=49, "
        "int coll=-1) -> ()");
  m.def("fc1_wgrad_adam(Tensor dz, Tensor a2, Tensor h, Tensor dlog, Tensor(a!) gW3, Tensor(b!) gb3, Tensor(c!) gW4, "
        "Tensor(d!) gb4, int roles, Tensor? dz_w3, Tensor? a2_w3, Tensor(e!) p3, Tensor(f!) m3, Tensor(g!) v3, "
        "Tensor(h!) shadow3, Tensor state, float lr, float b1, float b2, float eps, float grad_scale, int rule, "
        "bool write_grad=False, int jt_lo=0, int jt_hi=49, int coll=-1) -> ()");
  m.def("fc1_dgrad(Tensor dz, Tensor w3bf, Tensor a2, Tensor(a!) g2) -> ()");
  m.def("conv2_wgrad_groups(int B) -> int", &mihvd::conv2_wgrad_groups);
  m.def("conv2_bwd(Tensor g2, Tensor idx2, Tensor a1, Tensor w2bf, Tensor x, Tensor? rows, Tensor? state, Tensor idx1, "
        "Tensor(a!) slab, Tensor(b!) cpart, Tensor(c!)? g1=None, int coll=-1) -> ()");
  m.def("conv2_wgrad_reduce(Tensor slab, Tensor cpart, int B, Tensor(a!) gW2, Tensor(b!) gW1, Tensor(c!) gb1, "
        "Tensor(d!) gb2) -> ()");
  m.def("conv2_bwd_adam(Tensor g2, Tensor idx2, Tensor a1, Tensor w2bf, Tensor x, Tensor? rows, Tensor(s!) state, "
        "Tensor idx1, Tensor(a!) slab, Tensor(b!) cpart, Tensor(c!) p3, Tensor g3, Tensor(d!) m3, Tensor(e!) v3, "
        "Tensor(f!) shadow3, float lr, float b1, float b2, float eps, float grad_scale, int rule) -> ()");
  m.def("conv2_bwd_w3adam(Tensor g2, Tensor idx2, Tensor a1, Tensor w2bf, Tensor x, Tensor? rows, Tensor(s!) state, "
        "Tensor idx1, Tensor(a!) slab, Tensor(b!) cpart, Tensor dzT, Tensor a2T, Tensor(c!) p3, Tensor(d!) m3, "
        "Tensor(e!) v3, Tensor(f!) shadow3, Tensor(g!)? gW3, float lr, float b1, float b2, float eps, "
        "float grad_scale, int rule) -> ()");
  m.def("conv2_wgrad_reduce_adam(Tensor slab, Tensor cpart, int B, Tensor(a!) gW2, Tensor(b!) gW1, Tensor(c!) gb1, "
        "Tensor(d!) gb2, Tensor grads, Tensor(e!) p, Tensor(f!) m, Tensor(g!) v, Tensor(h!) shadow, Tensor(s!) state, "
        "int fc_lo, int w3_lo, float lr, float b1, float b2, float eps, float grad_scale, int rule) -> ()");
  m.def("conv2_bwd_adam_fold(Tensor g2, Tensor idx2, Tensor a1, Tensor w2bf, Tensor x, Tensor? rows, "
        "Tensor(s!) state, Tensor idx1, Tensor(a!) slab, Tensor(b!) cpart, Tensor(c!) gW2, Tensor(d!) gW1, "
        "Tensor(e!) gb1, Tensor(f!) gb2, Tensor grads, Tensor(g!) p, Tensor(h!) m, Tensor(i!) v, Tensor(j!) shadow, "
        "Tensor(k!) sync, int fc_lo, int w3_lo, float lr, float b1, float b2, float eps, float grad_scale, "
        "int rule) -> ()");
  m.def("adam_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? shadow, Tensor(e!)? state, "
        "int host_step, float lr, float b1, float b2, float eps, float grad_scale, int rule, int bump=1, "
        "Tensor? loss_scale=None, int max_blocks=0) -> ()");
  m.def("multi_tensor_adam(Tensor(a!)[] p, Tensor[] g, Tensor(b!)[] m, Tensor(c!)[] v, Tensor? step, int host_step, "
        "float lr, float b1, float b2, float eps, float weight_decay, bool decoupled, int rule, float grad_scale) -> ()");
  m.def("multi_tensor_sgd(Tensor(a!)[] p, Tensor[] g, Tensor(b!)[] bufs, float lr, float momentum, float dampening, "
        "float weight_decay, bool nesterov, bool first, float grad_scale) -> ()");
  m.def("bump_step_(Tensor(a!) step) -> ()");
  m.def("f32_conv1_fwd(Tensor x, Tensor? rows, Tensor? state, Tensor w1, Tensor b1, Tensor(a!) a1, Tensor(b!) idx1, "
        "Tensor? w2=None, Tensor(f!)? w2frag=None, int coll=-1, Tensor? xpre=None) -> ()");
  m.def("f32_prime_batch(Tensor x, Tensor labels, Tensor rows, Tensor state, Tensor(a!) xpre, Tensor(b!) ypre) -> ()");
  m.def("f32_conv2_fwd(Tensor a1, Tensor w2, Tensor b2, Tensor(a!) a2, Tensor(b!) idx2, Tensor? w2frag=None, int products=0) -> ()");
  m.def("f32_fc1_fwd(Tensor a2, Tensor w3, Tensor(a!) zpart, int products=0) -> ()");
  m.def("f32_head_fwd_bwd(Tensor zpart, Tensor b3, Tensor w4, Tensor b4, Tensor labels, Tensor? rows, "
        "Tensor(s!)? state, int seed, float rate, Tensor(a!) h, Tensor(b!) dz, Tensor(c!) dlog, Tensor(d!) stats, "
        "Tensor(e!)? stats_acc=None, Tensor? ypre=None) -> ()");
  m.def("f32_fc1_bwd(Tensor dz, Tensor a2, Tensor idx2, Tensor h, Tensor dlog, Tensor(w!) w3, Tensor(a!) dY2, "
        "Tensor(b!) db2p, Tensor(c!) gW3, Tensor(d!) gb3, Tensor(e!) gW4, Tensor(f!) gb4, Tensor(m!)? m3=None, "
        "Tensor(v!)? v3=None, Tensor? state=None, float lr=0., float beta1=0., float beta2=0., float eps=0., "
        "float grad_scale=1., int rule=0, bool store_w3=True, Tensor? px=None, Tensor? plabels=None, "
        "Tensor? prows=None, Tensor? pstate=None, Tensor(p!)? xpre=None, Tensor(q!)? ypre=None) -> ()");
  m.def("f32_factor_rows(Tensor a2c, Tensor dz, Tensor(a!)? out=None, Tensor(b!)? p=None, Tensor(c!)? m=None, "
        "Tensor(d!)? v=None, Tensor? state=None, float lr=0., float beta1=0., float beta2=0., float eps=0., "
        "float grad_scale=1., int rule=0) -> ()");
  m.def("f32_factor_full(Tensor a2, Tensor dz, int B, Tensor(a!)? out, Tensor(b!) p, Tensor(c!) m, Tensor(d!) v, "
        "Tensor state, float lr, float beta1, float beta2, float eps, float grad_scale, int rule) -> ()");
  m.def("f32_conv2_bwd(Tensor dY2, Tensor w2, Tensor a1, Tensor idx1, Tensor x, Tensor? rows, Tensor? state, "
        "Tensor(a!) cpart, Tensor(b!) slab, Tensor? w2frag=None, int products=0) -> ()");
  m.def("f32_conv_reduce(Tensor slab, Tensor cpart, Tensor db2p, Tensor(a!) gW2, Tensor(b!) gW1, Tensor(c!) gb1, "
        "Tensor(d!) gb2, Tensor(e!)? params=None, Tensor? grads=None, Tensor(f!)? m=None, Tensor(g!)? v=None, "
        "Tensor(s!)? state=None, int o_w1=0, int o_b1=0, int o_w2=0, int o_b2=0, int fc_lo=0, int fc_hi=0, "
        "float lr=0., float b1=0., float b2=0., float eps=0., float grad_scale=1., int rule=0) -> ()");
  m.def("f32_db2_rows(int B) -> int", &mihvd::f32_db2_rows);
  m.def("f32_stamps_enable(int n_blocks, int kernel=0) -> Tensor", &mihvd::f32_stamps_enable);
  m.def("f32_wgrad_groups(int B, int products=0) -> int", &mihvd::f32_wgrad_groups);
  m.def("f32_dgrad_blocks(int B, int products=0) -> int", &mihvd::f32_dgrad_blocks);
  m.def("conv_barrier_error(bool reset=True) -> int", &mihvd::conv_barrier_error);
  m.def("gather_cols_bf16(Tensor src, int col0, Tensor(a!) dst) -> ()");
  m.def("scale_cast_bf16(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("bf16_to_f32(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("scale_cast_f16(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("f16_to_f32(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("segment_dots(Tensor a, Tensor b, Tensor offs, int max_seg_len, Tensor(a!) out) -> ()");
  m.def("adasum_combine(Tensor a, Tensor b, Tensor offs, int max_seg_len, Tensor dots, Tensor(a!) out) -> ()");
  m.def("grad_check_(Tensor(a!)[] grads, Tensor(b!) ls, bool unscale) -> ()");
  m.def("update_scale_(Tensor(a!) ls, Tensor(b!) tracker, float growth, float backoff, int interval, "
        "float min_scale, Tensor(c!)? state=None) -> ()");
}

TORCH_LIBRARY_IMPL(mihvd, CUDA, m) {
  m.impl("conv1_fwd", &conv1_fwd_op);
  m.impl("conv2_fwd", &conv2_fwd_op);
  m.impl("conv12_fwd", &conv12_fwd_op);
  m.impl("fc1_bwd", &fc1_bwd_op);
  m.impl("fc1_fwd", &fc1_fwd_op);
  m.impl("head_fwd_bwd", &head_op);
  m.impl("conv1_fwd_f16", &conv1_fwd_f16_op);
  m.impl("conv2_fwd_f16", &conv2_fwd_f16_op);
  m.impl("conv12_fwd_f16", &conv12_fwd_f16_op);
  m.impl("fc1_fwd_f16", &fc1_fwd_f16_op);
  m.impl("head_fwd_bwd_f16", &head_f16_op);
  m.impl("fc1_bwd_f16", &fc1_bwd_f16_op);
  m.impl("conv2_bwd_f16", &conv2_bwd_f16_op);
  m.impl("fc1_wgrad", &fc1_wgrad_op);
  m.impl("fc1_wgrad_adam", &fc1_wgrad_adam_op);
  m.impl("fc1_dgrad", &fc1_dgrad_op);
  m.impl("conv2_bwd", &conv2_bwd_op);
  m.impl("conv2_wgrad_reduce", &conv2_wgrad_reduce_op);
  m.impl("conv2_bwd_adam", &conv2_bwd_adam_op);
  m.impl("conv2_bwd_w3adam", &conv2_bwd_w3adam_op);
  m.impl("conv2_wgrad_reduce_adam", &conv2_wgrad_reduce_adam_op);
  m.impl("conv2_bwd_adam_fold", &conv2_bwd_adam_fold_op);
  m.impl("adam_step", &adam_op);
  m.impl("gather_cols_bf16", &gather_cols_op);
  m.impl("multi_tensor_adam", &mt_adam_op);
  m.impl("multi_tensor_sgd", &mt_sgd_op);
  m.impl("bump_step_", &bump_step_op);
  m.impl("f32_conv1_fwd", &f32_conv1_op);
  m.impl("f32_prime_batch", &f32_prime_op);
  m.impl("f32_factor_rows", &f32_factor_rows_op);
  m.impl("f32_factor_full", &f32_factor_full_op);
  m.impl("f32_conv2_fwd", &f32_conv2_op);
  m.impl("f32_fc1_fwd", &f32_fc1_fwd_op);
  m.impl("f32_head_fwd_bwd", &f32_head_op);
  m.impl("f32_fc1_bwd", &f32_fc1_bwd_op);
  m.impl("f32_conv2_bwd", &f32_conv2_bwd_op);
  m.impl("f32_conv_reduce", &f32_conv_reduce_op);
  m.impl("scale_cast_bf16", &scale_cast_op);
  m.impl("bf16_to_f32", &bf16_to_f32_op);
  m.impl("scale_cast_f16", &scale_cast_f16_op);
  m.impl("f16_to_f32", &f16_to_f32_op);
  m.impl("segment_dots", &segment_dots_op);
  m.impl("adasum_combine", &adasum_combine_op);
  m.impl("grad_check_", &grad_check_op);
  m.impl("update_scale_", &update_scale_op);
}
