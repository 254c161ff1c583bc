// Collective negotiation engine (SURVEY.md §2.3 N1 background thread, N2 coordinator, N8 stall
// inspector). See control.h for the protocol overview.
//
// Store keys (under `prefix/`):
//   req_seq            global request counter (ADD gives every submission a unique, totally
//                      ordered sequence number across all ranks)
//   req/<seq>          "<rank>\x1f<name>\x1f<signature>" (a full request), or
//                      "<rank>\x1d<hex bit vector>" (response cache: every set bit i is a
//                      submission of the (name, signature) cached in slot i)
//   resp/<k>           the k-th response record: one or more
//                      "<generation>\x1f<name>\x1f<error>\x1f<slot>" entries joined by \x1e —
//                      collectives that became ready on all ranks in the same coordinator pass
//                      (slot: the pair's response-cache slot, -1 after an error). A record is a
//                      unit every rank sees identically, so it is also the unit inside which the
//                      executor may fuse tensors.
//   ack/<rank>         highest response index a rank has consumed (lets the coordinator delete)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <stdexcept>

#include "control.h"

namespace mihvd {

namespace {
using Clock = std::chrono::steady_clock;
constexpr double kPollS = 0.05;     // blocking-read granularity (stop latency)
constexpr int64_t kAckEvery = 256;  // responses between ack/<rank> updates

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t a = 0;
  for (;;) {
    size_t b = s.find(sep, a);
    if (b == std::string::npos) {
      out.push_back(s.substr(a));
      return out;
    }
    out.push_back(s.substr(a, b - a));
    a = b + 1;
  }
}

std::string bits_to_hex(const std::vector<uint8_t>& bits) {
  static const char* hx = "0123456789abcdef";
  std::string out;
  for (size_t i = 0; i < bits.size(); i += 4) {
    int v = 0;
    for (size_t j = 0; j < 4 && i + j < bits.size(); ++j) v |= (bits[i + j] ? 1 : 0) << j;
    out += hx[v];
  }
  return out;
}

std::vector<int> hex_to_slots(const std::string& hex) {
  std::vector<int> out;
  for (size_t i = 0; i < hex.size(); ++i) {
    const char c = hex[i];
    const int v = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : 0;
    for (int j = 0; j < 4; ++j)
      if (v & (1 << j)) out.push_back((int)(4 * i + j));
  }
  return out;
}

std::string ranks_str(const std::vector<int>& r) {
  std::ostringstream os;
  os << "[";
  for (size_t i = 0; i < r.size(); ++i) os << (i ? ", " : "") << r[i];
  os << "]";
  return os.str();
}
}  // namespace

Negotiator::Negotiator(const std::string& host, int port, int rank, int size, const std::string& prefix,
                       double cycle_s, double warn_s, double shutdown_s)
    : rank_(rank), size_(size), prefix_(prefix), cycle_s_(cycle_s), warn_s_(warn_s), shutdown_s_(shutdown_s) {
  if (size < 1 || rank < 0 || rank >= size) throw std::invalid_argument("Negotiator: bad rank/size");
  post_ = std::make_unique<StoreClient>(host, port, 60.0);
  resp_ = std::make_unique<StoreClient>(host, port, 60.0);
  if (rank_ == 0) {
    coord_ = std::make_unique<StoreClient>(host, port, 60.0);
    generation_of_rank_.resize(size_);
    coordinator_ = std::thread([this] { coordinator_loop(); });
  }
  engine_ = std::thread([this] { engine_loop(); });
  poster_ = std::thread([this] { poster_loop(); });
}

Negotiator::~Negotiator() { stop(); }

void Negotiator::stop() {
  if (stop_.exchange(true)) return;
  cv_.notify_all();
  if (poster_.joinable()) poster_.join();
  if (engine_.joinable()) engine_.join();
  if (coordinator_.joinable()) coordinator_.join();
}

void Negotiator::submit(const std::string& name, const std::string& signature) {
  for (const std::string* t : {&name, &signature})
    if (t->find('\x1f') != std::string::npos || t->find('\x1e') != std::string::npos)
      throw std::invalid_argument("Negotiator: names and signatures must not contain \\x1e or \\x1f");
  {
    std::lock_guard<std::mutex> g(mu_);
    outbox_.emplace_back(name, signature);
    sig_q_[name].push_back(signature);
  }
  submitted_.fetch_add(1);
  cv_.notify_all();
}

std::vector<Response> Negotiator::poll() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Response> out(ready_.begin(), ready_.end());
  ready_.clear();
  return out;
}

std::vector<Response> Negotiator::wait(double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  auto pred = [this] { return !ready_.empty() || stop_.load(); };
  if (timeout_s < 0) cv_.wait(lk, pred);
  else cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred);
  std::vector<Response> out(ready_.begin(), ready_.end());
  ready_.clear();
  return out;
}

// Every rank: the poster thread appends queued submissions to the global request log...
void Negotiator::poster_loop() {
  try {
    while (!stop_.load()) {
      std::deque<std::pair<std::string, std::string>> batch;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait_for(lk, std::chrono::duration<double>(kPollS), [this] { return !outbox_.empty() || stop_.load(); });
        batch.swap(outbox_);
      }
      if (batch.empty()) continue;
      // records in submission order; cached pairs accumulate in a bit vector that is flushed
      // before a full request and before a second submission of the same slot, so every rank's
      // per-name submission order survives
      std::vector<std::string> recs;
      std::vector<uint8_t> bits;
      bool any = false;
      auto flush_bits = [&] {
        if (!any) return;
        recs.push_back(std::to_string(rank_) + '\x1d' + bits_to_hex(bits));
        std::fill(bits.begin(), bits.end(), 0);
        any = false;
      };
      for (auto& e : batch) {
        int slot = -1;
        {
          std::lock_guard<std::mutex> g(mu_);
          auto it = rank_cache_.find(e.first + '\x1f' + e.second);
          if (it != rank_cache_.end()) slot = it->second;
        }
        if (slot < 0) {
          flush_bits();
          recs.push_back(std::to_string(rank_) + '\x1f' + e.first + '\x1f' + e.second);
          continue;
        }
        if ((size_t)slot >= bits.size()) bits.resize(slot + 1, 0);
        if (bits[slot]) flush_bits();
        bits[slot] = 1;
        any = true;
        cache_hits_.fetch_add(1);
      }
      flush_bits();
      const int64_t last = post_->add(key("req_seq"), (int64_t)recs.size());
      int64_t seq = last - (int64_t)recs.size() + 1;
      for (auto& r : recs) post_->set(key("req/" + std::to_string(seq++)), r);
      records_posted_.fetch_add((int64_t)recs.size());
    }
  } catch (const std::exception& e) {
    if (!stop_.load()) std::fprintf(stderr, "[mihvd negotiator rank %d] poster thread stopped: %s\n", rank_, e.what());
  }
}

// ...and the engine thread reads the response log (identical on every rank) into the ready queue.
void Negotiator::engine_loop() {
  int64_t next_resp = 1;
  try {
    while (!stop_.load()) {
      std::string v;
      if (!resp_->try_get(key("resp/" + std::to_string(next_resp)), kPollS, &v)) continue;
      auto recs = split(v, '\x1e');
      {
        std::lock_guard<std::mutex> g(mu_);
        for (const auto& rec : recs) {
          auto f = split(rec, '\x1f');
          Response r;
          r.generation = std::stoll(f.at(0));
          r.name = f.at(1);
          r.error = f.size() > 2 ? f[2] : "";
          r.batch = next_resp;
          // learn the pair's cache slot (the signature is the one this rank submitted: a pair
          // with an error is never cached)
          auto q = sig_q_.find(r.name);
          if (q != sig_q_.end() && !q->second.empty()) {
            const std::string sig = std::move(q->second.front());
            q->second.pop_front();
            if (q->second.empty()) sig_q_.erase(q);
            if (f.size() > 3 && r.error.empty()) {
              const int slot = std::stoi(f[3]);
              if (slot >= 0) rank_cache_[r.name + '\x1f' + sig] = slot;
            }
          }
          ready_.push_back(std::move(r));
        }
      }
      responded_.fetch_add((int64_t)recs.size());
      cv_.notify_all();
      if (next_resp % kAckEvery == 0) resp_->set(key("ack/" + std::to_string(rank_)), std::to_string(next_resp));
      ++next_resp;
    }
  } catch (const std::exception& e) {
    if (!stop_.load()) std::fprintf(stderr, "[mihvd negotiator rank %d] engine thread stopped: %s\n", rank_, e.what());
  }
}

std::vector<StallEntry> Negotiator::stalled(double older_than_s) const {
  std::vector<StallEntry> out;
  std::lock_guard<std::mutex> g(mu_);
  auto now = Clock::now();
  for (const auto& kv : pending_) {
    const Pending& p = kv.second;
    double age = std::chrono::duration<double>(now - p.first_seen).count();
    if (age < older_than_s) continue;
    StallEntry e;
    e.name = kv.first.first;
    e.generation = kv.first.second;
    e.age_s = age;
    for (int r = 0; r < size_; ++r) (p.have[r] ? e.ready_ranks : e.missing_ranks).push_back(r);
    out.push_back(std::move(e));
  }
  return out;
}

// Rank 0: consume the request log in order, count (name, generation) submissions, publish the
// collectives that every rank has submitted, and report stalls.
void Negotiator::coordinator_loop() {
  int64_t next_req = 1, next_out = 1, deleted_upto = 0;
  auto last_scan = Clock::now();
  try {
    while (!stop_.load()) {
      std::string v;
      // One pass: the first request (blocking up to kPollS), then every request already in the
      // log; everything that completes in the pass is published as one response record.
      std::string record;
      int n_in_pass = 0;
      while (n_in_pass < 1024 &&
             coord_->try_get(key("req/" + std::to_string(next_req)), n_in_pass == 0 ? kPollS : 0.0, &v)) {
        ++n_in_pass;
        coord_->del(key("req/" + std::to_string(next_req)));
        ++next_req;
        // a full request, or a bit vector of cached (name, signature) slots
        std::vector<std::pair<int, std::pair<std::string, std::string>>> subs;
        const size_t bv = v.find('\x1d');
        if (bv != std::string::npos) {
          const int r = std::stoi(v.substr(0, bv));
          std::lock_guard<std::mutex> g(mu_);
          for (int slot : hex_to_slots(v.substr(bv + 1)))
            if (slot < (int)coord_slots_.size()) subs.push_back({r, coord_slots_[slot]});
        } else {
          auto f = split(v, '\x1f');
          subs.push_back({std::stoi(f.at(0)), {f.at(1), f.size() > 2 ? f[2] : ""}});
        }
        for (auto& sub : subs) {
        const int r = sub.first;
        const std::string& name = sub.second.first;
        const std::string& sig = sub.second.second;
        std::string publish;
        {
          std::lock_guard<std::mutex> g(mu_);
          const int64_t gen = generation_of_rank_.at(r)[name]++;
          auto k = std::make_pair(name, gen);
          auto it = pending_.find(k);
          if (it == pending_.end()) {
            Pending p;
            p.signature = sig;
            p.have.assign(size_, 0);
            p.first_seen = Clock::now();
            it = pending_.emplace(k, std::move(p)).first;
          } else if (sig != it->second.signature && it->second.error.empty()) {
            it->second.error = "mismatched collective '" + name + "': rank " + std::to_string(r) + " submitted [" + sig +
                               "], another rank [" + it->second.signature + "]";
          }
          Pending& p = it->second;
          p.have[r] = 1;
          if (++p.count == size_) {
            int slot = -1;
            if (p.error.empty()) {
              const std::string ck = name + '\x1f' + p.signature;
              auto cit = coord_cache_.find(ck);
              if (cit == coord_cache_.end()) {
                cit = coord_cache_.emplace(ck, (int)coord_slots_.size()).first;
                coord_slots_.push_back({name, p.signature});
              }
              slot = cit->second;
            }
            publish = std::to_string(gen) + '\x1f' + name + '\x1f' + p.error + '\x1f' + std::to_string(slot);
            pending_.erase(it);
          }
        }
        if (!publish.empty()) {
          if (!record.empty()) record += '\x1e';
          record += publish;
        }
        }
      }
      if (!record.empty()) coord_->set(key("resp/" + std::to_string(next_out++)), record);
      auto now = Clock::now();
      if (std::chrono::duration<double>(now - last_scan).count() >= 0.25) {
        last_scan = now;
        // stall inspector: report each pending (name, generation) once past warn_s
        std::vector<std::string> msgs;
        bool abort_now = false;
        {
          std::lock_guard<std::mutex> g(mu_);
          for (auto& kv : pending_) {
            Pending& p = kv.second;
            double age = std::chrono::duration<double>(now - p.first_seen).count();
            if (warn_s_ > 0 && age >= warn_s_ && !p.warned) {
              p.warned = true;
              std::vector<int> ready, missing;
              for (int rr = 0; rr < size_; ++rr) (p.have[rr] ? ready : missing).push_back(rr);
              char age_s[32];
              std::snprintf(age_s, sizeof(age_s), "%.1f", age);
              msgs.push_back("collective '" + kv.first.first + "' (generation " + std::to_string(kv.first.second) +
                             ") was submitted by ranks " + ranks_str(ready) + " but not by ranks " + ranks_str(missing) +
                             " for " + age_s + " s");
            }
            if (shutdown_s_ > 0 && age >= shutdown_s_) abort_now = true;
          }
        }
        for (auto& m : msgs) {
          warnings_.fetch_add(1);
          std::fprintf(stderr, "[mihvd stall inspector] %s\n", m.c_str());
        }
        if (abort_now) {
          std::fprintf(stderr, "[mihvd stall inspector] stall exceeded %.0f s: aborting the job\n", shutdown_s_);
          std::fflush(stderr);
          std::_Exit(134);
        }
        // garbage-collect responses every rank has acknowledged
        int64_t min_ack = next_out - 1;
        for (int rr = 0; rr < size_ && min_ack > deleted_upto; ++rr) {
          std::string a;
          min_ack = coord_->try_get(key("ack/" + std::to_string(rr)), 0.0, &a) ? std::min<int64_t>(min_ack, (int64_t)std::stoll(a)) : 0;
        }
        for (; deleted_upto < min_ack; ++deleted_upto) coord_->del(key("resp/" + std::to_string(deleted_upto + 1)));
      }
    }
  } catch (const std::exception& e) {
    if (!stop_.load()) std::fprintf(stderr, "[mihvd negotiator] coordinator thread stopped: %s\n", e.what());
  }
}

}  // namespace mihvd
