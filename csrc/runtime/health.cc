// Communicator health monitor: the failure-detection half of SURVEY.md §5.3 / §5.8.
//
// The reference relies on MPI's abort semantics (horovod/tensorflow-mnist.yaml:17-38: mpirun tears
// the whole job down when a rank fails). With RCCL a failure can instead surface asynchronously:
// a peer dies or a link errors, and the communicator reports it through ncclCommGetAsyncError while
// the other ranks sit in a collective that will never complete. This monitor owns that path in
// native code: a background thread polls the async-error state of every attached RCCL
// communicator (symbols resolved from the librccl the process already loaded, so the communicator
// pointer and the library agree); on an error it reports it, aborts every attached communicator
// (ncclCommAbort: in-flight kernels are cancelled instead of spinning) and terminates the process
// with a non-zero code, so mihvdrun / mpirun kill the remaining ranks promptly.
//
// The direct-xGMI plane has no communicator: its device-side phase barriers mirror a timeout into a
// host-coherent error word (csrc/kernels/xgmi.hip), which the same thread watches (watch_word), so
// a peer that never arrives ends the job within one poll interval instead of at the next host sync.
//
// inject_error() (driven by MIHVD_FAULT="collerr:...") sets the same error from a test, which is how
// the path is exercised on CPU-only machines.
#include <dlfcn.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>

#include "runtime.h"

namespace mihvd {

namespace {
// ncclResult_t values of rccl.h (RCCL 2.27): 0 success, 7 in progress (non-blocking init)
constexpr int kNcclSuccess = 0;
constexpr int kNcclInProgress = 7;
constexpr int kWordError = 6;  // a watched error word: reported as a remote error (a peer never arrived)
const char* fallback_name(int code) {
  switch (code) {
    case 1: return "unhandled HIP error";
    case 2: return "system error";
    case 3: return "internal error";
    case 4: return "invalid argument";
    case 5: return "invalid usage";
    case 6: return "remote error (a peer failed)";
    default: return "error";
  }
}
}  // namespace

HealthMonitor::HealthMonitor(int rank, double poll_s, int exit_code)
    : rank_(rank), poll_s_(poll_s > 0 ? poll_s : 0.5), exit_code_(exit_code) {}

HealthMonitor::~HealthMonitor() { stop(); }

bool HealthMonitor::attach_rccl(uintptr_t comm, const std::string& lib_path) {
  std::lock_guard<std::mutex> lk(mu_);
  if (comm == 0) return false;
  if (lib_ == nullptr) {
    // the library that created the communicator is already mapped: take a reference to it
    void* h = dlopen(lib_path.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (h == nullptr) h = dlopen(lib_path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) return false;
    get_err_ = reinterpret_cast<GetErrFn>(dlsym(h, "ncclCommGetAsyncError"));
    abort_ = reinterpret_cast<AbortFn>(dlsym(h, "ncclCommAbort"));
    err_str_ = reinterpret_cast<ErrStrFn>(dlsym(h, "ncclGetErrorString"));
    if (get_err_ == nullptr) {
      dlclose(h);
      get_err_ = nullptr;
      abort_ = nullptr;
      err_str_ = nullptr;
      return false;
    }
    lib_ = h;
  }
  comms_.push_back(reinterpret_cast<void*>(comm));
  return true;
}

void HealthMonitor::detach_rccl(uintptr_t comm) {
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t i = 0; i < comms_.size(); ++i)
    if (comms_[i] == reinterpret_cast<void*>(comm)) {
      comms_.erase(comms_.begin() + (ptrdiff_t)i);
      return;
    }
}

void HealthMonitor::inject_error(int code, const std::string& what) {
  std::lock_guard<std::mutex> lk(mu_);
  injected_ = code;
  injected_what_ = what;
  cv_.notify_all();
}

void HealthMonitor::watch_word(uintptr_t addr, const std::string& label) {
  std::lock_guard<std::mutex> lk(mu_);
  if (addr == 0) return;
  for (auto& w : words_)
    if (w.first == reinterpret_cast<const uint32_t*>(addr)) return;
  words_.emplace_back(reinterpret_cast<const uint32_t*>(addr), label);
}

void HealthMonitor::unwatch_word(uintptr_t addr) {
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t i = 0; i < words_.size(); ++i)
    if (words_[i].first == reinterpret_cast<const uint32_t*>(addr)) {
      words_.erase(words_.begin() + (ptrdiff_t)i);
      return;
    }
}

int64_t HealthMonitor::num_words() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int64_t)words_.size();
}

int64_t HealthMonitor::num_comms() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int64_t)comms_.size();
}

void HealthMonitor::start() {
  std::lock_guard<std::mutex> lk(mu_);
  if (running_) return;
  running_ = true;
  stop_ = false;
  thread_ = std::thread([this] { loop(); });
}

void HealthMonitor::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!running_) return;
    stop_ = true;
    cv_.notify_all();
  }
  if (thread_.joinable()) thread_.join();
  std::lock_guard<std::mutex> lk(mu_);
  running_ = false;
}

// One poll over every attached communicator (and the injected error). Returns the first error.
int HealthMonitor::poll_once(std::string* what) {
  std::lock_guard<std::mutex> lk(mu_);
  polls_.fetch_add(1);
  if (injected_ != kNcclSuccess) {
    if (what) *what = "injected (" + injected_what_ + ")";
    return injected_;
  }
  for (void* c : comms_) {
    int e = kNcclSuccess;
    if (get_err_ != nullptr && get_err_(c, &e) == kNcclSuccess && e != kNcclSuccess && e != kNcclInProgress) {
      if (what) {
        char buf[64];
        std::snprintf(buf, sizeof(buf), "communicator %p", c);
        *what = buf;
      }
      return e;
    }
  }
  for (const auto& w : words_) {
    // written by device code with system-scope stores into host-coherent memory
    const uint32_t v = __atomic_load_n(w.first, __ATOMIC_ACQUIRE);
    if (v != 0u) {
      if (what) {
        char buf[32];
        std::snprintf(buf, sizeof(buf), " (error word %#x)", v);
        *what = w.second + buf;
      }
      return kWordError;
    }
  }
  return kNcclSuccess;
}

void HealthMonitor::fail(int code, const std::string& what) {
  error_.store(code);
  const char* name = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (err_str_ != nullptr) name = err_str_(code);
  }
  std::fprintf(stderr,
               "[rank %d] mihvd health: collective error %d (%s) on %s; aborting the communicator(s) and "
               "exiting with %d so the launcher tears the job down\n",
               rank_, code, name ? name : fallback_name(code), what.c_str(), exit_code_);
  std::fflush(stderr);
  if (!abort_process_) return;
  std::vector<void*> comms;
  AbortFn ab = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu_);
    comms = comms_;
    ab = abort_;
  }
  if (ab != nullptr)
    for (void* c : comms) ab(c);
  std::fflush(stdout);
  _exit(exit_code_);
}

void HealthMonitor::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::duration<double>(poll_s_), [this] { return stop_ || injected_ != kNcclSuccess; });
    if (stop_) break;
    lk.unlock();
    std::string what;
    const int e = poll_once(&what);
    if (e != kNcclSuccess) {
      fail(e, what);
      lk.lock();
      break;  // (only reached with abort_process_ off)
    }
    lk.lock();
  }
}

}  // namespace mihvd
