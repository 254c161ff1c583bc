// Multi-tensor fused optimizers for arbitrary PyTorch models (mihvd.optim.FusedAdam / FusedSGD).
//
// The fused MNIST step updates one flat buffer (optim.hip). Models trained through the generic
// DistributedOptimizer keep one tensor per parameter, so these kernels take a table of up to
// MT_T tensors per launch and map blocks to (tensor, 32K-element chunk) pairs: the whole update of
// a model is a handful of launches instead of ~7 foreach kernels per optimizer step, and the
// optimizer step count can live on the device, so the update can be captured in a HIP graph
// together with forward, backward and the RCCL allreduces (mihvd/graphs.py).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include <vector>

#include "common.h"

namespace mihvd {

constexpr int MT_T = 24;          // tensors per launch
constexpr int MT_B = 320;         // blocks per launch
constexpr int64_t MT_CHUNK = 32768;

struct MTTable {
  float* p[MT_T];
  const float* g[MT_T];
  float* s1[MT_T];
  float* s2[MT_T];
  int64_t n[MT_T];
  uint8_t vec[MT_T];   // 16-byte aligned and n % 4 == 0: float4 path
  int16_t tidx[MT_B];
  int32_t chunk[MT_B];
};

struct AdamHyper {
  float lr, b1, b2, eps, wd, gscale;
  int rule;        // 0: TF1 (eps outside the bias-corrected sqrt), 1: torch
  int decoupled;   // AdamW
  const int64_t* step_dev;  // device step counter (optional, read *after* the host bump)
  int64_t step_host;
};

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamCoef& c, float wd,
                                          float lr, int decoupled) {
  if (wd != 0.f) {
    if (decoupled) p -= lr * wd * p;
    else g = fmaf(wd, p, g * c.gscale) / c.gscale;  // L2: on the unscaled gradient
  }
  adam1(p, m, v, g, c);
}

__global__ void __launch_bounds__(256) mt_adam_kernel(MTTable tt, AdamHyper h) {
  const int t = tt.tidx[blockIdx.x];
  const int64_t c0 = (int64_t)tt.chunk[blockIdx.x] * MT_CHUNK;
  const int64_t n = tt.n[t];
  const int64_t c1 = min(c0 + MT_CHUNK, n);
  const float step = (float)(h.step_dev ? *h.step_dev : h.step_host);
  const AdamCoef c = adam_coef(step, h.lr, h.b1, h.b2, h.eps, h.gscale, h.rule);
  float* p = tt.p[t];
  const float* g = tt.g[t];
  float* m = tt.s1[t];
  float* v = tt.s2[t];
  if (tt.vec[t]) {
    for (int64_t i = (c0 >> 2) + threadIdx.x; i < (c1 >> 2); i += 256) {
      float4 pp = reinterpret_cast<float4*>(p)[i];
      float4 gg = reinterpret_cast<const float4*>(g)[i];
      float4 mm = reinterpret_cast<float4*>(m)[i];
      float4 vv = reinterpret_cast<float4*>(v)[i];
      adam_elem(pp.x, mm.x, vv.x, gg.x, c, h.wd, h.lr, h.decoupled);
      adam_elem(pp.y, mm.y, vv.y, gg.y, c, h.wd, h.lr, h.decoupled);
      adam_elem(pp.z, mm.z, vv.z, gg.z, c, h.wd, h.lr, h.decoupled);
      adam_elem(pp.w, mm.w, vv.w, gg.w, c, h.wd, h.lr, h.decoupled);
      reinterpret_cast<float4*>(p)[i] = pp;
      reinterpret_cast<float4*>(m)[i] = mm;
      reinterpret_cast<float4*>(v)[i] = vv;
    }
  } else {
    for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
      float pp = p[i], mm = m[i], vv = v[i];
      adam_elem(pp, mm, vv, g[i], c, h.wd, h.lr, h.decoupled);
      p[i] = pp;
      m[i] = mm;
      v[i] = vv;
    }
  }
}

struct SgdHyper {
  float lr, momentum, dampening, wd, gscale;
  int nesterov, first;  // first: the momentum buffer starts as the gradient (torch semantics)
};

__device__ __forceinline__ void sgd_elem(float& p, float& buf, float g, const SgdHyper& h, bool has_buf) {
  float d = g * h.gscale;
  if (h.wd != 0.f) d = fmaf(h.wd, p, d);
  if (has_buf) {
    buf = h.first ? d : fmaf(h.momentum, buf, (1.f - h.dampening) * d);
    d = h.nesterov ? fmaf(h.momentum, buf, d) : buf;
  }
  p -= h.lr * d;
}

__global__ void __launch_bounds__(256) mt_sgd_kernel(MTTable tt, SgdHyper h) {
  const int t = tt.tidx[blockIdx.x];
  const int64_t c0 = (int64_t)tt.chunk[blockIdx.x] * MT_CHUNK;
  const int64_t n = tt.n[t];
  const int64_t c1 = min(c0 + MT_CHUNK, n);
  float* p = tt.p[t];
  const float* g = tt.g[t];
  float* b = tt.s1[t];
  const bool has_buf = b != nullptr;
  float dummy = 0.f;
  for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
    float pp = p[i];
    float& bb = has_buf ? b[i] : dummy;
    sgd_elem(pp, bb, g[i], h, has_buf);
    p[i] = pp;
  }
}

// ------------------------------------------------------------------------------------------ //
template <typename Launch>
static void for_each_batch(const std::vector<at::Tensor>& p, const std::vector<at::Tensor>& g,
                           const std::vector<at::Tensor>* s1, const std::vector<at::Tensor>* s2, Launch launch) {
  const size_t nt = p.size();
  TORCH_CHECK(g.size() == nt && (!s1 || s1->size() == nt) && (!s2 || s2->size() == nt), "multi-tensor: list lengths");
  MTTable tt{};
  int ntab = 0, nblk = 0;
  auto flush = [&]() {
    if (nblk > 0) launch(tt, nblk);
    tt = MTTable{};
    ntab = 0;
    nblk = 0;
  };
  for (size_t i = 0; i < nt; ++i) {
    const int64_t n = p[i].numel();
    if (n == 0) continue;
    for (const at::Tensor* x : {&p[i], &g[i]})
      TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kFloat && x->is_contiguous() && x->numel() == n,
                  "multi-tensor optimizer: contiguous fp32 GPU tensors of equal size expected");
    if (s1) TORCH_CHECK((*s1)[i].scalar_type() == at::kFloat && (*s1)[i].is_contiguous() && (*s1)[i].numel() == n, "state 1");
    if (s2) TORCH_CHECK((*s2)[i].scalar_type() == at::kFloat && (*s2)[i].is_contiguous() && (*s2)[i].numel() == n, "state 2");
    const int64_t chunks = (n + MT_CHUNK - 1) / MT_CHUNK;
    if (ntab == MT_T) flush();
    tt.p[ntab] = p[i].data_ptr<float>();
    tt.g[ntab] = g[i].data_ptr<float>();
    tt.s1[ntab] = s1 ? (*s1)[i].data_ptr<float>() : nullptr;
    tt.s2[ntab] = s2 ? (*s2)[i].data_ptr<float>() : nullptr;
    tt.n[ntab] = n;
    bool vec = n % 4 == 0;
    for (float* q : {tt.p[ntab], const_cast<float*>(tt.g[ntab]), tt.s1[ntab], tt.s2[ntab]})
      if (q && ((uintptr_t)q & 15)) vec = false;
    tt.vec[ntab] = vec ? 1 : 0;
    for (int64_t c = 0; c < chunks; ++c) {
      if (nblk == MT_B) {
        // keep the current tensor as entry 0 of the next launch
        MTTable keep{};
        keep.p[0] = tt.p[ntab];
        keep.g[0] = tt.g[ntab];
        keep.s1[0] = tt.s1[ntab];
        keep.s2[0] = tt.s2[ntab];
        keep.n[0] = tt.n[ntab];
        keep.vec[0] = tt.vec[ntab];
        launch(tt, nblk);
        tt = keep;
        ntab = 0;
        nblk = 0;
      }
      tt.tidx[nblk] = (int16_t)ntab;
      tt.chunk[nblk] = (int32_t)c;
      ++nblk;
    }
    ++ntab;
  }
  flush();
}

void multi_tensor_adam(std::vector<at::Tensor> p, std::vector<at::Tensor> g, std::vector<at::Tensor> m,
                       std::vector<at::Tensor> v, const c10::optional<at::Tensor>& step, int64_t host_step, double lr,
                       double b1, double b2, double eps, double weight_decay, bool decoupled, int64_t rule,
                       double grad_scale) {
  AdamHyper h{(float)lr, (float)b1, (float)b2, (float)eps, (float)weight_decay, (float)grad_scale, (int)rule,
              decoupled ? 1 : 0, nullptr, host_step};
  if (step.has_value() && step->defined()) {
    TORCH_CHECK(step->is_cuda() && step->scalar_type() == at::kLong && step->numel() >= 1, "multi_tensor_adam: step");
    h.step_dev = step->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(host_step >= 1, "multi_tensor_adam: step must be >= 1");
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  for_each_batch(p, g, &m, &v, [&](const MTTable& tt, int nblk) { mt_adam_kernel<<<nblk, 256, 0, stream>>>(tt, h); });
}

void multi_tensor_sgd(std::vector<at::Tensor> p, std::vector<at::Tensor> g, std::vector<at::Tensor> bufs, double lr,
                      double momentum, double dampening, double weight_decay, bool nesterov, bool first,
                      double grad_scale) {
  SgdHyper h{(float)lr, (float)momentum, (float)dampening, (float)weight_decay, (float)grad_scale, nesterov ? 1 : 0,
             first ? 1 : 0};
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const bool has = !bufs.empty();
  for_each_batch(p, g, has ? &bufs : nullptr, nullptr,
                 [&](const MTTable& tt, int nblk) { mt_sgd_kernel<<<nblk, 256, 0, stream>>>(tt, h); });
}

// device step counter: += 1 (graph-capturable optimizer step count)
__global__ void bump_kernel(int64_t* s) { s[0] += 1; }
void bump_step_(at::Tensor& step) {
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kLong, "bump_step_: int64 GPU tensor");
  bump_kernel<<<1, 1, 0, c10::hip::getCurrentHIPStream().stream()>>>(step.data_ptr<int64_t>());
}

}  // namespace mihvd
