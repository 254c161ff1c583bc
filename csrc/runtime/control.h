// mihvd control plane: bootstrap key-value store and the collective-negotiation engine.
//
// SURVEY.md §2.3 N10 / N1 / N2 / N8. The reference reaches these through Open MPI and Horovod's C++
// core (`hvd.init()` horovod/tensorflow_mnist.py:90, every allreduce of `hvd.DistributedOptimizer`
// :133); here they are native host code next to the RCCL data plane:
//
//   * StoreServer / StoreClient - a TCP key-value store (the rendezvous server that `mihvdrun`
//     hosts, like horovodrun's). It backs `torch.distributed.init_process_group(store=...)`, i.e.
//     it carries the ncclUniqueId exchange of RCCL, and it is the control channel of the
//     negotiation engine. Blocking reads (GET/WAIT) are parked on the server and answered when the
//     key appears or the deadline passes, so clients never poll.
//   * Negotiator - Horovod's background thread + coordinator (operations.cc / controller.cc):
//     every rank submits the names of the collectives it is ready to run in whatever order its
//     program produces them; rank 0's coordinator thread reads the global, totally ordered
//     request log from the store, counts submissions per (name, generation), checks that every
//     rank submitted the same signature (op, dtype, shape) and publishes a response log of names
//     that are ready on all ranks. Every rank's engine thread reads the response log, so all
//     ranks launch their collectives in the same order — no deadlock when ranks enqueue tensors
//     in different orders. The coordinator also knows which ranks are missing for each pending
//     tensor: that is Horovod's stall inspector message ("ranks [..] did not submit X").
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "slot_agreement.h"

namespace mihvd {

// ---------------------------------------------------------------------------------------------
// Key-value store (TCP). Wire format: frame = u32 length | u8 op | payload; strings are
// u32 length + bytes, integers little-endian i64. Responses: u32 length | u8 status | payload.
// ---------------------------------------------------------------------------------------------
enum StoreOp : uint8_t {
  kSet = 1, kGet = 2, kAdd = 3, kCheck = 4, kWait = 5, kCompareSet = 6, kDelete = 7,
  kNumKeys = 8, kAppend = 9, kPing = 10,
};
enum StoreStatus : uint8_t { kOk = 0, kTimeout = 1, kError = 2 };

class StoreServer {
 public:
  // port 0 picks an ephemeral port (see port()). host "" / "0.0.0.0" listens on every interface.
  StoreServer(const std::string& host, int port);
  ~StoreServer();
  int port() const { return port_; }
  int64_t num_keys() const;
  int64_t num_connections() const { return nconn_.load(); }
  void stop();

 private:
  struct Conn;
  struct Waiter;
  void loop();
  void handle(Conn& c, uint8_t op, const std::string& payload);
  void reply(Conn& c, uint8_t status, const std::string& payload);
  void wake_waiters();
  bool ready_for(const Waiter& w) const;
  void answer(Waiter& w, bool timed_out);

  int listen_fd_ = -1;
  int wake_fd_[2] = {-1, -1};
  int port_ = 0;
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> nconn_{0};
  mutable std::mutex mu_;  // guards kv_ for num_keys() from other threads
  std::unordered_map<std::string, std::string> kv_;
  std::vector<std::unique_ptr<Conn>> conns_;
  std::vector<Waiter> waiters_;
  std::thread thread_;
};

class StoreClient {
 public:
  // Connects (retrying until connect_timeout_s) to a StoreServer.
  StoreClient(const std::string& host, int port, double connect_timeout_s = 60.0);
  ~StoreClient();
  void set(const std::string& key, const std::string& value);
  // Blocks until the key exists; throws std::runtime_error on timeout (timeout_s < 0: forever).
  std::string get(const std::string& key, double timeout_s = -1.0);
  // Like get() but returns false on timeout instead of throwing.
  bool try_get(const std::string& key, double timeout_s, std::string* value);
  int64_t add(const std::string& key, int64_t delta);
  bool check(const std::vector<std::string>& keys);
  bool wait(const std::vector<std::string>& keys, double timeout_s = -1.0);
  // torch.distributed semantics: set `desired` if the current value equals `expected` (a missing
  // key matches an empty `expected`); returns the value after the operation.
  std::string compare_set(const std::string& key, const std::string& expected, const std::string& desired);
  bool del(const std::string& key);
  void append(const std::string& key, const std::string& value);
  int64_t num_keys();
  void close();
  const std::string& host() const { return host_; }
  int port() const { return port_; }

 private:
  uint8_t request(uint8_t op, const std::string& payload, std::string* out);
  int fd_ = -1;
  std::string host_;
  int port_;
  std::mutex mu_;
};

// ---------------------------------------------------------------------------------------------
// Negotiation engine
// ---------------------------------------------------------------------------------------------
struct StallEntry {
  std::string name;
  int64_t generation;
  double age_s;
  std::vector<int> ready_ranks;
  std::vector<int> missing_ranks;
};

struct Response {
  std::string name;
  int64_t generation = 0;
  std::string error;  // non-empty: signature mismatch (the collective must not be launched)
  int64_t batch = 0;  // response-record index: names published together (a fusion group candidate)
};

class Negotiator {
 public:
  // `prefix` namespaces the store keys (one negotiation domain per process set).
  // warn_s: the coordinator logs tensors that some ranks submitted and others did not for longer
  //         than this (0 disables); shutdown_s > 0 aborts the job (exit 134) after that long.
  Negotiator(const std::string& host, int port, int rank, int size, const std::string& prefix,
             double cycle_s, double warn_s, double shutdown_s);
  ~Negotiator();
  // Thread-safe, non-blocking: queue a collective named `name` with a consistency signature.
  void submit(const std::string& name, const std::string& signature);
  // Responses in the global order (identical on every rank). Non-blocking / blocking variants.
  std::vector<Response> poll();
  std::vector<Response> wait(double timeout_s);
  // Coordinator view (rank 0 only; empty elsewhere): tensors waiting for some ranks.
  std::vector<StallEntry> stalled(double older_than_s) const;
  int64_t submitted() const { return submitted_.load(); }
  int64_t responses() const { return responded_.load(); }
  int64_t warnings() const { return warnings_.load(); }
  // response cache: submissions that went out as a bit of a cached-slot vector, and request
  // records written to the store (full requests + bit-vector records)
  int64_t cache_hits() const { return cache_hits_.load(); }
  int64_t records_posted() const { return records_posted_.load(); }
  void stop();

 private:
  void poster_loop();
  void engine_loop();
  void coordinator_loop();
  std::string key(const std::string& k) const { return prefix_ + "/" + k; }

  int rank_, size_;
  std::string prefix_;
  double cycle_s_, warn_s_, shutdown_s_;  // cycle_s_: reserved (responses are pushed, not polled)
  std::unique_ptr<StoreClient> post_, resp_, coord_;
  std::atomic<bool> stop_{false};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<std::string, std::string>> outbox_;
  std::deque<Response> ready_;
  std::atomic<int64_t> submitted_{0}, responded_{0}, warnings_{0}, cache_hits_{0}, records_posted_{0};
  // Response cache (Horovod's response_cache.cc): the coordinator gives every (name, signature)
  // it has published without error a slot; every rank learns the slots from the responses. A
  // later submission of a cached pair is posted as one bit of a per-batch slot bit vector
  // ("<rank>\x1d<hex bits>") instead of a full request record, so steady-state negotiation costs
  // one store write per poster batch, not one per tensor. A pair whose signature changed misses
  // the cache and goes out in full, so the coordinator still sees (and reports) the mismatch.
  std::unordered_map<std::string, int> rank_cache_;   // every rank: name \x1f sig -> slot
  // every rank: signatures of its outstanding submissions per name, in submission order (the
  // responses of one name come back in generation order, so the front is the response's)
  std::unordered_map<std::string, std::deque<std::string>> sig_q_;
  std::unordered_map<std::string, int> coord_cache_;  // rank 0: name \x1f sig -> slot
  std::vector<std::pair<std::string, std::string>> coord_slots_;  // rank 0: slot -> (name, sig)

  // coordinator state (rank 0)
  struct Pending {
    std::string signature;
    std::vector<char> have;
    int count = 0;
    std::chrono::steady_clock::time_point first_seen;
    bool warned = false;
    std::string error;
  };
  std::map<std::pair<std::string, int64_t>, Pending> pending_;                // (name, generation)
  std::vector<std::unordered_map<std::string, int64_t>> generation_of_rank_;  // per rank, per name
  std::thread poster_, engine_, coordinator_;
};

// ---------------------------------------------------------------------------------------------
// The native engine's control plane over the TCP store (engine.cpp runs it over RCCL)
// ---------------------------------------------------------------------------------------------
// CtrlTransport of SlotAgreement over the key-value store: round r of a collective is every rank's
// value under <prefix>/r<r>/<rank>; a rank reads all of them (parked blocking gets) and deletes its
// own value of round r - 2 (every rank has read it by then: it finished round r - 1).
class StoreCtrlTransport final : public CtrlTransport {
 public:
  StoreCtrlTransport(const std::string& host, int port, int rank, int world, const std::string& prefix,
                     double timeout_s = 60.0);
  int world() const override { return world_; }
  void allreduce_sum_i32(int32_t* v, int n) override;
  void allgather_i32(const int32_t* mine, int K, int32_t* out) override;
  int64_t rounds() const { return round_; }
  int64_t bytes_posted() const { return bytes_; }

 private:
  std::vector<std::string> exchange(const std::string& mine);
  StoreClient client_;
  int rank_, world_;
  std::string prefix_;
  double timeout_s_;
  int64_t round_ = 0, bytes_ = 0;
};

// The engine's negotiation (SlotAgreement) driven over StoreCtrlTransport: the CPU-testable form of
// engine.cpp's cycle (tests/test_distributed_cpu.py::test_engine_slot_agreement_over_store).
class EngineNegotiation {
 public:
  EngineNegotiation(const std::string& host, int port, int rank, int world, const std::string& prefix, int cap,
                    int announce_k);
  void want(uint32_t h) { agree_.want(h); }
  int slot(uint32_t h) const { return agree_.slot(h); }
  int num_slots() const { return agree_.num_slots(); }
  std::vector<int32_t> negotiate(const std::vector<int>& pending, bool stop) {
    return agree_.negotiate(ctrl_, pending, stop);
  }
  std::vector<uint32_t> announce_round() { return agree_.announce_round(ctrl_); }
  // the ready slots of a summed control vector, grouped for fusion (-1 ends a group)
  std::vector<int64_t> plan(const std::vector<int32_t>& summed, const std::vector<int64_t>& bytes,
                            const std::vector<int64_t>& key, int64_t threshold, std::vector<int>* partial) const;
  int64_t announces() const { return agree_.announces(); }
  int64_t max_fresh() const { return agree_.max_fresh(); }
  int64_t rounds() const { return ctrl_.rounds(); }

 private:
  SlotAgreement agree_;
  StoreCtrlTransport ctrl_;
};

}  // namespace mihvd
