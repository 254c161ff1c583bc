// torch.library registration of the mihvd HIP kernels: torch.ops.mihvd.<name>.
// All ops launch on the current HIP stream and allocate nothing, so they can be captured into a
// HIP graph by torch.cuda.graph.
#include <ATen/ATen.h>
#include <torch/library.h>

namespace mihvd {
void conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1);
void conv2_fwd(const at::Tensor& a1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2);
void fc1_fwd(const at::Tensor& a2, const at::Tensor& w3bf, at::Tensor& zpart);
void head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                  const at::Tensor& labels, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                  int64_t seed, double rate, at::Tensor& h, at::Tensor& dz, at::Tensor& dlog, at::Tensor& stats);
void fc1_bwd(const at::Tensor& dz, const at::Tensor& w3bf, const at::Tensor& a2, const at::Tensor& h,
             const at::Tensor& dlog, at::Tensor& dap, at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4,
             at::Tensor& gb2, at::Tensor& gW1, at::Tensor& gb1);
int64_t conv2_wgrad_groups(int64_t B);
void conv2_bwd(const at::Tensor& dap, const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a1,
               const at::Tensor& w2bf, at::Tensor& g1, at::Tensor& slab, at::Tensor& gb2);
void conv1_wgrad(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                 const at::Tensor& g1, const at::Tensor& idx1, const at::Tensor& slab, at::Tensor& gW1, at::Tensor& gb1,
                 at::Tensor& gW2);
void adam_step(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, const c10::optional<at::Tensor>& shadow,
               const c10::optional<at::Tensor>& state, int64_t host_step, double lr, double b1, double b2, double eps,
               double grad_scale, int64_t rule);
void scale_cast_bf16(const at::Tensor& src, at::Tensor& dst, double scale);
void bf16_to_f32(const at::Tensor& src, at::Tensor& dst, double scale);
}  // namespace mihvd

static void conv1_fwd_op(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                         const at::Tensor& w1, const at::Tensor& b1, at::Tensor a1, at::Tensor idx1) {
  mihvd::conv1_fwd(x, rows, state, w1, b1, a1, idx1);
}
static void conv2_fwd_op(const at::Tensor& a1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor a2, at::Tensor idx2) {
  mihvd::conv2_fwd(a1, w2, b2, a2, idx2);
}
static void fc1_fwd_op(const at::Tensor& a2, const at::Tensor& w3, at::Tensor zpart) { mihvd::fc1_fwd(a2, w3, zpart); }
static void head_op(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                    const at::Tensor& labels, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                    int64_t seed, double rate, at::Tensor h, at::Tensor dz, at::Tensor dlog, at::Tensor stats) {
  mihvd::head_fwd_bwd(zpart, b3, w4, b4, labels, rows, state, seed, rate, h, dz, dlog, stats);
}
static void fc1_bwd_op(const at::Tensor& dz, const at::Tensor& w3, const at::Tensor& a2, const at::Tensor& h,
                       const at::Tensor& dlog, at::Tensor dap, at::Tensor gW3, at::Tensor gb3, at::Tensor gW4, at::Tensor gb4,
                       at::Tensor gb2, at::Tensor gW1, at::Tensor gb1) {
  mihvd::fc1_bwd(dz, w3, a2, h, dlog, dap, gW3, gb3, gW4, gb4, gb2, gW1, gb1);
}
static void conv2_bwd_op(const at::Tensor& dap, const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& a1,
                         const at::Tensor& w2, at::Tensor g1, at::Tensor slab, at::Tensor gb2) {
  mihvd::conv2_bwd(dap, a2, idx2, a1, w2, g1, slab, gb2);
}
static void conv1_wgrad_op(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                           const at::Tensor& g1, const at::Tensor& idx1, const at::Tensor& slab, at::Tensor gW1,
                           at::Tensor gb1, at::Tensor gW2) {
  mihvd::conv1_wgrad(x, rows, state, g1, idx1, slab, gW1, gb1, gW2);
}
static void adam_op(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, const c10::optional<at::Tensor>& shadow,
                    const c10::optional<at::Tensor>& state, int64_t host_step, double lr, double b1, double b2, double eps,
                    double grad_scale, int64_t rule) {
  mihvd::adam_step(p, g, m, v, shadow, state, host_step, lr, b1, b2, eps, grad_scale, rule);
}
static void scale_cast_op(const at::Tensor& src, at::Tensor dst, double scale) { mihvd::scale_cast_bf16(src, dst, scale); }
static void bf16_to_f32_op(const at::Tensor& src, at::Tensor dst, double scale) { mihvd::bf16_to_f32(src, dst, scale); }

TORCH_LIBRARY(mihvd, m) {
  m.def("conv1_fwd(Tensor x, Tensor? rows, Tensor? state, Tensor w1, Tensor b1, Tensor(a!) a1, Tensor(b!) idx1) -> ()");
  m.def("conv2_fwd(Tensor a1, Tensor w2bf, Tensor b2, Tensor(a!) a2, Tensor(b!) idx2) -> ()");
  m.def("fc1_fwd(Tensor a2, Tensor w3bf, Tensor(a!) zpart) -> ()");
  m.def("head_fwd_bwd(Tensor zpart, Tensor b3, Tensor w4, Tensor b4, Tensor labels, Tensor? rows, Tensor(s!)? state, "
        "int seed, float rate, Tensor(a!) h, Tensor(b!) dz, Tensor(c!) dlog, Tensor(d!) stats) -> ()");
  m.def("fc1_bwd(Tensor dz, Tensor w3bf, Tensor a2, Tensor h, Tensor dlog, Tensor(a!) dap, Tensor(b!) gW3, "
        "Tensor(c!) gb3, Tensor(d!) gW4, Tensor(e!) gb4, Tensor(f!) gb2, Tensor(g!) gW1, Tensor(h!) gb1) -> ()");
  m.def("conv2_wgrad_groups(int B) -> int", &mihvd::conv2_wgrad_groups);
  m.def("conv2_bwd(Tensor dap, Tensor a2, Tensor idx2, Tensor a1, Tensor w2bf, Tensor(a!) g1, Tensor(b!) slab, "
        "Tensor(c!) gb2) -> ()");
  m.def("conv1_wgrad(Tensor x, Tensor? rows, Tensor? state, Tensor g1, Tensor idx1, Tensor slab, Tensor(a!) gW1, "
        "Tensor(b!) gb1, Tensor(c!) gW2) -> ()");
  m.def("adam_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? shadow, Tensor(e!)? state, "
        "int host_step, float lr, float b1, float b2, float eps, float grad_scale, int rule) -> ()");
  m.def("scale_cast_bf16(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def("bf16_to_f32(Tensor src, Tensor(a!) dst, float scale) -> ()");
}

TORCH_LIBRARY_IMPL(mihvd, CUDA, m) {
  m.impl("conv1_fwd", &conv1_fwd_op);
  m.impl("conv2_fwd", &conv2_fwd_op);
  m.impl("fc1_fwd", &fc1_fwd_op);
  m.impl("head_fwd_bwd", &head_op);
  m.impl("fc1_bwd", &fc1_bwd_op);
  m.impl("conv2_bwd", &conv2_bwd_op);
  m.impl("conv1_wgrad", &conv1_wgrad_op);
  m.impl("adam_step", &adam_op);
  m.impl("scale_cast_bf16", &scale_cast_op);
  m.impl("bf16_to_f32", &bf16_to_f32_op);
}
