// Slot agreement of the native collective engine (csrc/kernels/engine.cpp), transport-agnostic.
//
// Horovod's coordinator makes every rank launch its collectives in the same
// order even when the ranks enqueue tensors in different orders (the reference's DistributedOptimizer
// allreduces, horovod/tensorflow_mnist.py:133, go through it). The engine does this without a
// coordinator rank: a signature (name, dtype, numel, op; 32-bit hash) gets a SLOT every rank agrees
// on, and each cycle ONE sum-allreduce of a control vector tells every rank which slots are ready
// everywhere:
//
//   [0] ranks asking to stop with nothing pending   [1] ranks with unannounced signatures
//   [2 .. 2+S)      1 if this rank has work pending in slot s
//   [2+S .. 2+2S)   the slot's hash if pending here (0 otherwise): a consistency check
//
// When [1] > 0 an all-gather of up to K unannounced hashes per rank follows; every rank appends the
// sorted union of the hashes that have no slot yet (engine_new_slot_order), so the slot table is
// identical on every rank by construction, whatever order each rank enqueued in. A rank with more
// than K new signatures announces the rest in later cycles.
//
// The transport is what differs: the engine runs these two collectives on its RCCL control
// communicator (small device buffers on a control stream); the CPU tests run the very same code over
// the TCP key-value store (StoreCtrlTransport, csrc/runtime/engine_ctrl.cc) with 2..8 processes.
#pragma once

#include <algorithm>
#include <cstdint>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace mihvd {

// 32-bit FNV-1a of a collective's signature "name|dtype|numel|op" (0 is reserved: "nothing").
inline uint32_t engine_fnv32(const std::string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) h = (h ^ c) * 16777619u;
  return h == 0 ? 1u : h;
}

// The control plane's two collectives (every rank calls them in the same order).
struct CtrlTransport {
  virtual ~CtrlTransport() = default;
  virtual int world() const = 0;
  // v[0, n) summed over every rank, in place
  virtual void allreduce_sum_i32(int32_t* v, int n) = 0;
  // out[world * K] = every rank's K entries, in rank order
  virtual void allgather_i32(const int32_t* mine, int K, int32_t* out) = 0;
};

// A failure every rank detects identically (computed from the same summed / gathered data).
struct ConsistentControlError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Slot agreement (the announce step): `gathered` holds world x K announced hashes (0 = empty
// entry). Returns the hashes that get new slots, in the order every rank appends them: the sorted
// union of the announced hashes that have no slot yet. A pure function of data every rank holds.
inline std::vector<uint32_t> engine_new_slot_order(const int32_t* gathered, int world, int K,
                                                   const std::unordered_set<uint32_t>& assigned) {
  std::set<uint32_t> fresh;
  for (int i = 0; i < world * K; ++i) {
    const uint32_t h = (uint32_t)gathered[i];
    if (h != 0 && assigned.count(h) == 0) fresh.insert(h);
  }
  return std::vector<uint32_t>(fresh.begin(), fresh.end());
}

// Planning step: given the summed control vector, the slots' hashes and sizes / fuse keys, return
// the ready slots grouped for fusion (-1 ends a group), or an error on a signature mismatch.
inline std::vector<int64_t> engine_plan_groups(const int32_t* sum, int nslot, int world,
                                               const std::vector<uint32_t>& hash, const std::vector<int64_t>& bytes,
                                               const std::vector<int64_t>& key, int64_t threshold,
                                               std::vector<int>* partial, std::string* error) {
  std::vector<int64_t> out;
  int64_t cur_bytes = 0, cur_key = -1;
  bool open = false;
  for (int s = 0; s < nslot; ++s) {
    const int cnt = sum[2 + s];
    if (cnt == 0) continue;
    if (cnt < world) {
      if (partial) partial->push_back(s);
      continue;
    }
    const uint32_t hs = (uint32_t)sum[2 + nslot + s];
    if (hs != (uint32_t)((uint32_t)world * hash[s])) {
      if (error) *error = "slot " + std::to_string(s) + ": ranks enqueued different collectives (name/dtype/size/op)";
      return {};
    }
    const bool big = bytes[s] > threshold;
    if (open && (big || key[s] != cur_key || cur_bytes + bytes[s] > threshold)) {
      out.push_back(-1);
      open = false;
    }
    out.push_back(s);
    if (big) {
      out.push_back(-1);
      continue;
    }
    if (!open) {
      open = true;
      cur_bytes = 0;
      cur_key = key[s];
    }
    cur_bytes += bytes[s];
  }
  if (open) out.push_back(-1);
  return out;
}

// One rank's view of the slot table and its unannounced signatures.
class SlotAgreement {
 public:
  SlotAgreement(int world, int cap, int announce_k = 64) : world_(world), cap_(cap), K_(announce_k) {}

  int world() const { return world_; }
  int cap() const { return cap_; }
  int announce_k() const { return K_; }
  int num_slots() const { return (int)hash_.size(); }
  uint32_t hash_of(int s) const { return hash_[s]; }
  const std::vector<uint32_t>& hashes() const { return hash_; }
  // the agreed slot of a signature, or -1
  int slot(uint32_t h) const {
    auto it = slot_of_.find(h);
    return it == slot_of_.end() ? -1 : it->second;
  }
  // a local signature without a slot: announce it (once) in the coming cycles
  void want(uint32_t h) {
    if (slot(h) >= 0 || std::find(announce_.begin(), announce_.end(), h) != announce_.end()) return;
    announce_.push_back(h);
  }
  bool has_announce() const { return !announce_.empty(); }
  int64_t announces() const { return announces_; }
  int64_t max_fresh() const { return max_fresh_; }

  // The negotiation allreduce: `pending` = the slots with work pending on this rank, `stop` = this
  // rank asks to stop with nothing pending. Returns the summed control vector [2 + 2 cap].
  std::vector<int32_t> negotiate(CtrlTransport& t, const std::vector<int>& pending, bool stop) {
    std::vector<int32_t> v(2 + 2 * (size_t)cap_, 0);
    v[0] = stop ? 1 : 0;
    v[1] = announce_.empty() ? 0 : 1;
    for (int s : pending) {
      v[2 + s] = 1;
      v[2 + cap_ + s] = (int32_t)hash_[s];
    }
    t.allreduce_sum_i32(v.data(), (int)v.size());
    return v;
  }

  // The announce round (when the summed [1] > 0): all-gather up to K unannounced hashes per rank
  // and append the fresh ones as new slots (returned in slot order).
  std::vector<uint32_t> announce_round(CtrlTransport& t) {
    std::vector<int32_t> mine(K_, 0), all((size_t)world_ * K_, 0);
    for (int i = 0; i < K_ && i < (int)announce_.size(); ++i) mine[i] = (int32_t)announce_[i];
    t.allgather_i32(mine.data(), K_, all.data());
    std::unordered_set<uint32_t> assigned(hash_.begin(), hash_.end());
    const auto fresh = engine_new_slot_order(all.data(), world_, K_, assigned);
    if ((int)hash_.size() + (int)fresh.size() > cap_)
      throw ConsistentControlError("more than " + std::to_string(cap_) +
                                   " distinct collectives across the ranks (MIHVD_ENGINE_SLOTS)");
    for (uint32_t h : fresh) {
      slot_of_[h] = (int)hash_.size();
      hash_.push_back(h);
      announce_.erase(std::remove(announce_.begin(), announce_.end(), h), announce_.end());
    }
    ++announces_;
    max_fresh_ = std::max<int64_t>(max_fresh_, (int64_t)fresh.size());
    return fresh;
  }

 private:
  int world_, cap_, K_;
  std::vector<uint32_t> hash_;               // slot -> hash
  std::unordered_map<uint32_t, int> slot_of_;
  std::vector<uint32_t> announce_;           // local signatures without a slot, in enqueue order
  int64_t announces_ = 0, max_fresh_ = 0;
};

}  // namespace mihvd
