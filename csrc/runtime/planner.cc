// Fusion-buffer bucket planner + in-order readiness controller.
// Capability parity: Horovod tensor fusion (HOROVOD_FUSION_THRESHOLD, default 64 MiB) and the
// coordinator's cross-rank ordering guarantee, which the reference relies on through
// hvd.DistributedOptimizer (horovod/tensorflow_mnist.py:133, tensorflow_mnist_gpu.py:137-138).
#include <algorithm>
#include <map>
#include <sstream>
#include <stdexcept>
#include <tuple>

#include "runtime.h"

namespace mihvd {

BucketPlan plan_buckets(const std::vector<TensorSpec>& specs, const std::vector<int>& order,
                        int64_t threshold_bytes, int64_t align_bytes) {
  if (align_bytes <= 0) align_bytes = 1;
  BucketPlan plan;
  const int n = static_cast<int>(specs.size());
  plan.tensor_bucket.assign(n, -1);
  plan.tensor_offset.assign(n, 0);
  // One open bucket per (dtype, device) key; a bucket is closed when the next tensor would push
  // it past the threshold. Bucket ids are assigned at creation, so release order follows the
  // order in which the first member of each bucket becomes ready.
  std::map<std::pair<int, int>, int> open;
  std::vector<int64_t> bytes;
  for (int idx : order) {
    if (idx < 0 || idx >= n) throw std::out_of_range("plan_buckets: bad tensor index");
    if (plan.tensor_bucket[idx] != -1) throw std::invalid_argument("plan_buckets: duplicate index");
    const TensorSpec& s = specs[idx];
    const auto key = std::make_pair(s.dtype, s.device);
    const int64_t align_el = std::max<int64_t>(1, align_bytes / std::max(1, s.elem_size));
    const int64_t tbytes = s.numel * s.elem_size;
    auto it = open.find(key);
    int b = -1;
    if (it != open.end()) {
      b = it->second;
      const int64_t aligned_end = ((plan.numel[b] + align_el - 1) / align_el * align_el) * s.elem_size;
      if (threshold_bytes > 0 && bytes[b] > 0 && aligned_end + tbytes > threshold_bytes) b = -1;
    }
    if (b == -1) {
      b = static_cast<int>(plan.members.size());
      plan.members.emplace_back();
      plan.offsets.emplace_back();
      plan.numel.push_back(0);
      plan.dtype.push_back(s.dtype);
      plan.device.push_back(s.device);
      bytes.push_back(0);
      open[key] = b;
    }
    int64_t off = (plan.numel[b] + align_el - 1) / align_el * align_el;
    plan.members[b].push_back(idx);
    plan.offsets[b].push_back(off);
    plan.tensor_bucket[idx] = b;
    plan.tensor_offset[idx] = off;
    plan.numel[b] = off + s.numel;
    bytes[b] = plan.numel[b] * s.elem_size;
  }
  // Pad every bucket to the alignment so the vectorised pack/unpack kernels never straddle.
  for (size_t b = 0; b < plan.numel.size(); ++b) {
    int esz = specs[plan.members[b][0]].elem_size;
    int64_t align_el = std::max<int64_t>(1, align_bytes / std::max(1, esz));
    plan.numel[b] = (plan.numel[b] + align_el - 1) / align_el * align_el;
  }
  for (int i = 0; i < n; ++i)
    if (plan.tensor_bucket[i] == -1) throw std::invalid_argument("plan_buckets: tensor not in order");
  return plan;
}

Controller::Controller(std::vector<int> tensor_bucket, int num_buckets, int passes_per_step)
    : tensor_bucket_(std::move(tensor_bucket)), num_buckets_(num_buckets),
      passes_(std::max(1, passes_per_step)) {
  bucket_size_.assign(num_buckets_, 0);
  for (int b : tensor_bucket_) {
    if (b < 0 || b >= num_buckets_) throw std::out_of_range("Controller: bad bucket id");
    bucket_size_[b]++;
  }
  reset();
}

void Controller::reset() {
  remaining_ = bucket_size_;
  countdown_.assign(tensor_bucket_.size(), passes_);
  next_launch_ = 0;
}

std::vector<int> Controller::mark_ready(int tensor_idx) {
  if (tensor_idx < 0 || tensor_idx >= static_cast<int>(tensor_bucket_.size()))
    throw std::out_of_range("Controller::mark_ready: bad tensor index");
  if (countdown_[tensor_idx] <= 0) {
    std::ostringstream os;
    os << "gradient " << tensor_idx << " was computed more than backward_passes_per_step="
       << passes_ << " times before synchronize(); call optimizer.step() or synchronize() "
       << "between passes";
    throw std::runtime_error(os.str());
  }
  std::vector<int> out;
  if (--countdown_[tensor_idx] > 0) return out;
  const int b = tensor_bucket_[tensor_idx];
  remaining_[b]--;
  while (next_launch_ < num_buckets_ && remaining_[next_launch_] == 0) out.push_back(next_launch_++);
  return out;
}

std::vector<int> Controller::flush() {
  std::vector<int> out;
  while (next_launch_ < num_buckets_) out.push_back(next_launch_++);
  return out;
}

uint64_t fnv1a64(const std::string& s, uint64_t h) {
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ULL;
  }
  return h;
}

uint64_t tensor_signature(const std::vector<std::string>& names,
                          const std::vector<std::vector<int64_t>>& shapes,
                          const std::vector<std::string>& dtypes) {
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < names.size(); ++i) {
    h = fnv1a64(names[i], h);
    h = fnv1a64("|", h);
    if (i < shapes.size())
      for (int64_t d : shapes[i]) h = fnv1a64(std::to_string(d) + ",", h);
    if (i < dtypes.size()) h = fnv1a64(dtypes[i], h);
    h = fnv1a64(";", h);
  }
  return h;
}

}  // namespace mihvd
