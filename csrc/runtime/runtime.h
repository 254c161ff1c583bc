// mihvd native runtime: the host-side control plane of the data-parallel engine.
//
// This is the MI355X-native equivalent of the pieces of Horovod's C++ core that the reference
// relies on implicitly: the reference only *calls* them through
// `hvd.DistributedOptimizer` (horovod/tensorflow_mnist.py:133) and `hvd.init()` (:90).
//
//   * BucketPlanner  - static fusion-buffer layout (N3 "tensor fusion"): gradients are packed into
//                      flat, 256-byte aligned buckets, in reverse-registration (≈ backward) order.
//   * Controller     - replaces Horovod's coordinator negotiation (N2). Ranks run the same model, so
//                      readiness is tracked locally and buckets are released strictly in index
//                      order, which gives every rank the same collective order without a
//                      per-cycle network round trip. A 64-bit signature of (name, shape, dtype)
//                      is compared across ranks once, like Horovod's name/shape validation.
//   * Timeline       - Chrome-trace writer (N7, HOROVOD_TIMELINE) with a background writer thread.
//   * StallInspector - watchdog (N8, HOROVOD_STALL_CHECK_TIME_SECONDS): warns about collectives
//                      that have been outstanding too long and can hard-abort the process so the
//                      launcher tears the job down (mpirun semantics).
//   * FaultPlan      - env-driven fault injection (MIHVD_FAULT) used by the robustness tests.
//   * HealthMonitor  - RCCL async-error polling -> communicator abort -> non-zero exit.
//   * StepStats      - step-time accumulator for img/s and global_step/sec logging.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mihvd {

// ---------------------------------------------------------------------------------------------
// Bucket planning
// ---------------------------------------------------------------------------------------------
struct TensorSpec {
  int64_t numel = 0;
  int elem_size = 4;
  int dtype = 0;    // opaque dtype code chosen by the caller; buckets never mix codes
  int device = 0;   // opaque device code; buckets never mix devices
};

struct BucketPlan {
  std::vector<std::vector<int>> members;      // tensor indices per bucket (in pack order)
  std::vector<std::vector<int64_t>> offsets;  // element offset of each member inside the bucket
  std::vector<int64_t> numel;                 // padded bucket length in elements
  std::vector<int> dtype;
  std::vector<int> device;
  std::vector<int> tensor_bucket;             // tensor index -> bucket id
  std::vector<int64_t> tensor_offset;         // tensor index -> element offset in its bucket
};

// `order` lists tensor indices in the order they should be packed (normally reverse
// registration order, i.e. the order gradients become ready in backward).
BucketPlan plan_buckets(const std::vector<TensorSpec>& specs, const std::vector<int>& order,
                        int64_t threshold_bytes, int64_t align_bytes);

// ---------------------------------------------------------------------------------------------
// Readiness controller (in-order bucket release)
// ---------------------------------------------------------------------------------------------
class Controller {
 public:
  Controller(std::vector<int> tensor_bucket, int num_buckets, int passes_per_step);
  // Marks one gradient ready. Returns the bucket ids that may now be launched, in order.
  // Throws std::runtime_error if a gradient is produced more often than passes_per_step.
  std::vector<int> mark_ready(int tensor_idx);
  // Releases every bucket not yet launched (used by step()/synchronize() for unused params).
  std::vector<int> flush();
  void reset();
  int launched() const { return next_launch_; }
  int num_buckets() const { return num_buckets_; }
  int pending_in_bucket(int b) const { return remaining_[b]; }
  int passes_per_step() const { return passes_; }

 private:
  std::vector<int> tensor_bucket_;
  int num_buckets_;
  int passes_;
  std::vector<int> bucket_size_;
  std::vector<int> remaining_;
  std::vector<int> countdown_;
  int next_launch_ = 0;
};

uint64_t fnv1a64(const std::string& s, uint64_t seed = 1469598103934665603ULL);
uint64_t tensor_signature(const std::vector<std::string>& names,
                          const std::vector<std::vector<int64_t>>& shapes,
                          const std::vector<std::string>& dtypes);

// ---------------------------------------------------------------------------------------------
// Timeline (Chrome trace JSON array format)
// ---------------------------------------------------------------------------------------------
class Timeline {
 public:
  Timeline(const std::string& path, int rank);
  ~Timeline();
  void begin(const std::string& name, const std::string& cat, int64_t tid);
  void end(const std::string& name, const std::string& cat, int64_t tid);
  void complete(const std::string& name, const std::string& cat, int64_t tid, double ts_us,
                double dur_us);
  void instant(const std::string& name, const std::string& cat, int64_t tid);
  void counter(const std::string& name, double value);
  double now_us() const;
  void flush();
  void close();
  int64_t events_written() const { return written_.load(); }
  const std::string& path() const { return path_; }

 private:
  void push(std::string ev);
  void writer_loop();
  std::string path_;
  int rank_;
  std::chrono::steady_clock::time_point t0_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> queue_;
  bool stop_ = false;
  bool closed_ = false;
  bool first_ = true;
  std::atomic<int64_t> written_{0};
  std::atomic<int64_t> pushed_{0};
  std::FILE* fp_ = nullptr;
  std::thread writer_;
};

std::string json_escape(const std::string& s);

// ---------------------------------------------------------------------------------------------
// Stall inspector
// ---------------------------------------------------------------------------------------------
struct StallReport {
  std::string name;
  double age_s;
};

class StallInspector {
 public:
  // warn_s: age after which an outstanding op is reported once.
  // shutdown_s: if > 0, age after which the process is terminated with exit code 134 (abort
  //             semantics, so mihvdrun/mpirun kill the remaining ranks).
  StallInspector(double warn_s, double shutdown_s, double poll_s, int rank);
  ~StallInspector();
  int64_t submit(const std::string& name);
  void complete(int64_t id);
  std::vector<StallReport> outstanding(double older_than_s) const;
  int64_t num_outstanding() const;
  int64_t warnings_emitted() const { return warnings_.load(); }
  void start();
  void stop();
  bool stalled() const { return stalled_.load(); }
  void set_hard_abort(bool v) { hard_abort_ = v; }

 private:
  void loop();
  double warn_s_, shutdown_s_, poll_s_;
  int rank_;
  bool hard_abort_ = true;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<int64_t, std::pair<std::string, std::chrono::steady_clock::time_point>> ops_;
  std::unordered_map<int64_t, bool> warned_;
  int64_t next_id_ = 1;
  std::atomic<int64_t> warnings_{0};
  std::atomic<bool> stalled_{false};
  bool running_ = false;
  bool stop_ = false;
  std::thread thread_;
};

// ---------------------------------------------------------------------------------------------
// Fault injection: MIHVD_FAULT="kill:rank=1:step=50;delay:rank=0:step=3:ms=200"
// ---------------------------------------------------------------------------------------------
struct FaultAction {
  std::string kind;                       // kill | delay | hang | raise | nan
  int rank = -1;                          // -1 = every rank
  int64_t step = -1;                      // -1 = every step
  std::map<std::string, std::string> args;
};

class FaultPlan {
 public:
  explicit FaultPlan(const std::string& spec);
  std::vector<FaultAction> due(int rank, int64_t step) const;
  const std::vector<FaultAction>& actions() const { return actions_; }

 private:
  std::vector<FaultAction> actions_;
};

// ---------------------------------------------------------------------------------------------
// Communicator health monitor (health.cc): RCCL async-error polling -> abort -> non-zero exit
// ---------------------------------------------------------------------------------------------
class HealthMonitor {
 public:
  HealthMonitor(int rank, double poll_s, int exit_code);
  ~HealthMonitor();
  // Attach an RCCL communicator (ncclComm_t as an integer) created by the library at lib_path
  // (already loaded by the process). False if the library or its symbols are unavailable.
  bool attach_rccl(uintptr_t comm, const std::string& lib_path);
  void detach_rccl(uintptr_t comm);  // before the communicator is destroyed
  void inject_error(int code, const std::string& what);  // test hook (MIHVD_FAULT collerr)
  // Watch a 32-bit error word in host-visible memory (e.g. the xGMI plane's host-mapped timeout
  // mirror, csrc/kernels/xgmi.hip): nonzero is a collective failure like an RCCL async error.
  // The word must stay valid until unwatch_word().
  void watch_word(uintptr_t addr, const std::string& label);
  void unwatch_word(uintptr_t addr);
  int64_t num_words() const;
  int poll_once(std::string* what);                      // one check; the first error code or 0
  void start();
  void stop();
  int error() const { return error_.load(); }
  int64_t polls() const { return polls_.load(); }
  int64_t num_comms() const;
  void set_abort_process(bool v) { abort_process_ = v; }  // false: report only (tests)

 private:
  using GetErrFn = int (*)(void*, int*);
  using AbortFn = int (*)(void*);
  using ErrStrFn = const char* (*)(int);
  void loop();
  void fail(int code, const std::string& what);
  int rank_;
  double poll_s_;
  int exit_code_;
  bool abort_process_ = true;
  void* lib_ = nullptr;
  GetErrFn get_err_ = nullptr;
  AbortFn abort_ = nullptr;
  ErrStrFn err_str_ = nullptr;
  std::vector<void*> comms_;
  std::vector<std::pair<const uint32_t*, std::string>> words_;
  int injected_ = 0;
  std::string injected_what_;
  std::atomic<int> error_{0};
  std::atomic<int64_t> polls_{0};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool running_ = false;
  bool stop_ = false;
  std::thread thread_;
};

// ---------------------------------------------------------------------------------------------
// Step statistics (throughput logging)
// ---------------------------------------------------------------------------------------------
class StepStats {
 public:
  explicit StepStats(size_t window);
  void add(double ms);
  double mean() const;
  double percentile(double p) const;
  int64_t count() const { return count_; }
  void reset();

 private:
  size_t window_;
  std::deque<double> samples_;
  int64_t count_ = 0;
};

}  // namespace mihvd
