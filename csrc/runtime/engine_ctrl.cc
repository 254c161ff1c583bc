// The native engine's control plane over the TCP key-value store (control.h, slot_agreement.h).
//
// engine.cpp negotiates over its RCCL control communicator, which needs one GPU per rank; this
// transport carries the same two control collectives (the control-vector sum and the announce
// all-gather) through the store, so the engine's slot agreement runs in plain CPU processes: 2..8
// ranks enqueueing the same collectives in different orders, more than one announce round per
// cycle (tests/test_distributed_cpu.py).
#include <cstring>
#include <stdexcept>

#include "control.h"

namespace mihvd {

StoreCtrlTransport::StoreCtrlTransport(const std::string& host, int port, int rank, int world,
                                       const std::string& prefix, double timeout_s)
    : client_(host, port), rank_(rank), world_(world), prefix_(prefix), timeout_s_(timeout_s) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("StoreCtrlTransport: bad rank / world");
}

std::vector<std::string> StoreCtrlTransport::exchange(const std::string& mine) {
  const int64_t r = round_++;
  auto key = [&](int64_t rr, int p) { return prefix_ + "/r" + std::to_string(rr) + "/" + std::to_string(p); };
  client_.set(key(r, rank_), mine);
  bytes_ += (int64_t)mine.size();
  std::vector<std::string> all(world_);
  for (int p = 0; p < world_; ++p) all[p] = p == rank_ ? mine : client_.get(key(r, p), timeout_s_);
  if (r >= 2) client_.del(key(r - 2, rank_));
  return all;
}

void StoreCtrlTransport::allreduce_sum_i32(int32_t* v, int n) {
  const auto all = exchange(std::string(reinterpret_cast<const char*>(v), (size_t)n * 4));
  std::vector<int64_t> acc(n, 0);
  for (const auto& blob : all) {
    if ((int)blob.size() != n * 4) throw std::runtime_error("StoreCtrlTransport: control vectors of different lengths");
    const int32_t* x = reinterpret_cast<const int32_t*>(blob.data());
    for (int i = 0; i < n; ++i) acc[i] += x[i];
  }
  for (int i = 0; i < n; ++i) v[i] = (int32_t)(uint32_t)(uint64_t)acc[i];  // modular, like RCCL's int32 sum
}

void StoreCtrlTransport::allgather_i32(const int32_t* mine, int K, int32_t* out) {
  const auto all = exchange(std::string(reinterpret_cast<const char*>(mine), (size_t)K * 4));
  for (int p = 0; p < world_; ++p) {
    if ((int)all[p].size() != K * 4) throw std::runtime_error("StoreCtrlTransport: announce blocks of different lengths");
    std::memcpy(out + (size_t)p * K, all[p].data(), (size_t)K * 4);
  }
}

EngineNegotiation::EngineNegotiation(const std::string& host, int port, int rank, int world, const std::string& prefix,
                                     int cap, int announce_k)
    : agree_(world, cap, announce_k), ctrl_(host, port, rank, world, prefix) {}

std::vector<int64_t> EngineNegotiation::plan(const std::vector<int32_t>& summed, const std::vector<int64_t>& bytes,
                                             const std::vector<int64_t>& key, int64_t threshold,
                                             std::vector<int>* partial) const {
  const int S = agree_.cap();
  if ((int)summed.size() != 2 + 2 * S) throw std::invalid_argument("plan: summed must hold 2 + 2 cap entries");
  std::vector<uint32_t> hash(S, 0);
  std::vector<int64_t> b(S, 0), k(S, 0);
  for (int s = 0; s < agree_.num_slots(); ++s) {
    hash[s] = agree_.hash_of(s);
    if (s < (int)bytes.size()) b[s] = bytes[s];
    if (s < (int)key.size()) k[s] = key[s];
  }
  std::string err;
  auto out = engine_plan_groups(summed.data(), S, agree_.world(), hash, b, k, threshold, partial, &err);
  if (!err.empty()) throw ConsistentControlError(err);
  return out;
}

}  // namespace mihvd
