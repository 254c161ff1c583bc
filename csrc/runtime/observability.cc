// Timeline writer, stall inspector, fault plan and step statistics.
// Capability parity: Horovod Timeline (HOROVOD_TIMELINE), stall inspector
// (HOROVOD_STALL_CHECK_TIME_SECONDS / HOROVOD_STALL_SHUTDOWN_TIME_SECONDS) and the TF
// StepCounterHook's global_step/sec — none enabled in the reference job
// (horovod/tensorflow-mnist.yaml:17-38), all available here.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <unistd.h>

#include "runtime.h"

namespace mihvd {

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      case '\r': o += "\\r"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o += c;
        }
    }
  }
  return o;
}

// ------------------------------------------------------------------------------------------ //
Timeline::Timeline(const std::string& path, int rank)
    : path_(path), rank_(rank), t0_(std::chrono::steady_clock::now()) {
  fp_ = std::fopen(path.c_str(), "w");
  if (!fp_) throw std::runtime_error("Timeline: cannot open " + path);
  std::fputs("[\n", fp_);
  // Process-name metadata so chrome://tracing / Perfetto label each rank.
  std::ostringstream os;
  os << "{\"name\":\"process_name\",\"ph\":\"M\",\"pid\":" << rank_
     << ",\"args\":{\"name\":\"rank " << rank_ << "\"}}";
  push(os.str());
  writer_ = std::thread([this] { writer_loop(); });
}

Timeline::~Timeline() { close(); }

double Timeline::now_us() const {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0_).count();
}

void Timeline::push(std::string ev) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) return;
    queue_.push_back(std::move(ev));
    pushed_++;
  }
  cv_.notify_one();
}

static std::string event(const char* ph, const std::string& name, const std::string& cat,
                         int rank, int64_t tid, double ts) {
  std::ostringstream os;
  os.setf(std::ios::fixed);
  os.precision(3);
  os << "{\"name\":\"" << json_escape(name) << "\",\"cat\":\"" << json_escape(cat)
     << "\",\"ph\":\"" << ph << "\",\"ts\":" << ts << ",\"pid\":" << rank << ",\"tid\":" << tid;
  return os.str();
}

void Timeline::begin(const std::string& name, const std::string& cat, int64_t tid) {
  push(event("B", name, cat, rank_, tid, now_us()) + "}");
}
void Timeline::end(const std::string& name, const std::string& cat, int64_t tid) {
  push(event("E", name, cat, rank_, tid, now_us()) + "}");
}
void Timeline::complete(const std::string& name, const std::string& cat, int64_t tid,
                        double ts_us, double dur_us) {
  std::ostringstream os;
  os.setf(std::ios::fixed);
  os.precision(3);
  os << event("X", name, cat, rank_, tid, ts_us) << ",\"dur\":" << dur_us << "}";
  push(os.str());
}
void Timeline::instant(const std::string& name, const std::string& cat, int64_t tid) {
  push(event("i", name, cat, rank_, tid, now_us()) + ",\"s\":\"t\"}");
}
void Timeline::counter(const std::string& name, double value) {
  std::ostringstream os;
  os << event("C", name, "counter", rank_, 0, now_us()) << ",\"args\":{\"value\":" << value
     << "}}";
  push(os.str());
}

void Timeline::writer_loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
    std::deque<std::string> batch;
    batch.swap(queue_);
    lk.unlock();
    for (auto& ev : batch) {
      if (!first_) std::fputs(",\n", fp_);
      first_ = false;
      std::fputs(ev.c_str(), fp_);
      written_++;
    }
    std::fflush(fp_);
    lk.lock();
    if (stop_ && queue_.empty()) break;
  }
}

void Timeline::flush() {
  // Wait until the writer has drained everything pushed so far.
  const int64_t target = pushed_.load();
  for (int i = 0; i < 20000 && written_.load() < target; ++i) usleep(100);
}

void Timeline::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) return;
    closed_ = true;
    stop_ = true;
  }
  cv_.notify_one();
  if (writer_.joinable()) writer_.join();
  if (fp_) {
    std::fputs("\n]\n", fp_);
    std::fclose(fp_);
    fp_ = nullptr;
  }
}

// ------------------------------------------------------------------------------------------ //
StallInspector::StallInspector(double warn_s, double shutdown_s, double poll_s, int rank)
    : warn_s_(warn_s), shutdown_s_(shutdown_s), poll_s_(poll_s > 0 ? poll_s : 1.0), rank_(rank) {}

StallInspector::~StallInspector() { stop(); }

int64_t StallInspector::submit(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  int64_t id = next_id_++;
  ops_[id] = {name, std::chrono::steady_clock::now()};
  return id;
}

void StallInspector::complete(int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  ops_.erase(id);
  warned_.erase(id);
}

int64_t StallInspector::num_outstanding() const {
  std::lock_guard<std::mutex> g(mu_);
  return static_cast<int64_t>(ops_.size());
}

std::vector<StallReport> StallInspector::outstanding(double older_than_s) const {
  std::vector<StallReport> out;
  auto now = std::chrono::steady_clock::now();
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : ops_) {
    double age = std::chrono::duration<double>(now - kv.second.second).count();
    if (age >= older_than_s) out.push_back({kv.second.first, age});
  }
  std::sort(out.begin(), out.end(),
            [](const StallReport& a, const StallReport& b) { return a.age_s > b.age_s; });
  return out;
}

void StallInspector::start() {
  std::lock_guard<std::mutex> g(mu_);
  if (running_) return;
  running_ = true;
  stop_ = false;
  thread_ = std::thread([this] { loop(); });
}

void StallInspector::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!running_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  std::lock_guard<std::mutex> g(mu_);
  running_ = false;
}

void StallInspector::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::duration<double>(poll_s_), [this] { return stop_; });
    if (stop_) break;
    auto now = std::chrono::steady_clock::now();
    double worst = 0.0;
    std::vector<std::string> fresh;
    for (auto& kv : ops_) {
      double age = std::chrono::duration<double>(now - kv.second.second).count();
      worst = std::max(worst, age);
      if (age >= warn_s_ && !warned_[kv.first]) {
        warned_[kv.first] = true;
        std::ostringstream os;
        os << kv.second.first << " (" << static_cast<int>(age) << "s)";
        fresh.push_back(os.str());
      }
    }
    if (!fresh.empty()) {
      stalled_ = true;
      warnings_ += static_cast<int64_t>(fresh.size());
      std::ostringstream os;
      os << "[rank " << rank_ << "] mihvd stall inspector: collectives outstanding for more than "
         << warn_s_ << "s — one or more ranks have not submitted them (diverged control flow, a "
         << "dead rank or a hung device):";
      for (auto& f : fresh) os << "\n    " << f;
      std::cerr << os.str() << std::endl;
    }
    if (shutdown_s_ > 0 && worst >= shutdown_s_) {
      std::cerr << "[rank " << rank_ << "] mihvd stall inspector: stall exceeded "
                << shutdown_s_ << "s, shutting down (exit 134)" << std::endl;
      if (hard_abort_) std::_Exit(134);
      stalled_ = true;
    }
  }
}

// ------------------------------------------------------------------------------------------ //
static std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}

FaultPlan::FaultPlan(const std::string& spec) {
  for (auto& item : split(spec, ';')) {
    if (item.empty()) continue;
    auto parts = split(item, ':');
    FaultAction a;
    a.kind = parts[0];
    static const char* kinds[] = {"kill", "delay", "hang", "raise", "nan", "collerr"};
    bool ok = false;
    for (auto* k : kinds) ok |= (a.kind == k);
    if (!ok) throw std::invalid_argument("MIHVD_FAULT: unknown fault kind '" + a.kind + "'");
    for (size_t i = 1; i < parts.size(); ++i) {
      auto eq = parts[i].find('=');
      if (eq == std::string::npos)
        throw std::invalid_argument("MIHVD_FAULT: expected key=value, got '" + parts[i] + "'");
      std::string k = parts[i].substr(0, eq), v = parts[i].substr(eq + 1);
      if (k == "rank") a.rank = std::stoi(v);
      else if (k == "step") a.step = std::stoll(v);
      else a.args[k] = v;
    }
    actions_.push_back(a);
  }
}

std::vector<FaultAction> FaultPlan::due(int rank, int64_t step) const {
  std::vector<FaultAction> out;
  for (auto& a : actions_)
    if ((a.rank < 0 || a.rank == rank) && (a.step < 0 || a.step == step)) out.push_back(a);
  return out;
}

// ------------------------------------------------------------------------------------------ //
StepStats::StepStats(size_t window) : window_(std::max<size_t>(1, window)) {}
void StepStats::add(double ms) {
  samples_.push_back(ms);
  if (samples_.size() > window_) samples_.pop_front();
  count_++;
}
double StepStats::mean() const {
  if (samples_.empty()) return 0.0;
  double s = 0;
  for (double v : samples_) s += v;
  return s / samples_.size();
}
double StepStats::percentile(double p) const {
  if (samples_.empty()) return 0.0;
  std::vector<double> v(samples_.begin(), samples_.end());
  std::sort(v.begin(), v.end());
  double pos = std::min(1.0, std::max(0.0, p / 100.0)) * (v.size() - 1);
  size_t lo = static_cast<size_t>(std::floor(pos)), hi = static_cast<size_t>(std::ceil(pos));
  return v[lo] + (v[hi] - v[lo]) * (pos - lo);
}
void StepStats::reset() {
  samples_.clear();
  count_ = 0;
}

}  // namespace mihvd
