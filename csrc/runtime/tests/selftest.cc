// Native self-test of the host runtime, built without Python so it can run under AddressSanitizer /
// UndefinedBehaviorSanitizer and ThreadSanitizer (sanitizer builds of the host code;
// GPU sanitizers are not available on the MI355X pool). Exercises every multi-threaded component
// with real concurrency: the store server with many client threads, the negotiation engine with
// ranks as threads submitting in different orders, the timeline writer thread and the stall
// inspector thread. Exit code 0 = pass.
//
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -pthread csrc/runtime/*.cc selftest.cc
//   g++ -std=c++17 -O1 -g -fsanitize=thread -pthread ...            (tests/test_sanitizers_cpu.py)
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../control.h"
#include "../runtime.h"

using namespace mihvd;

#define CHECK(cond)                                                             \
  do {                                                                          \
    if (!(cond)) {                                                              \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

static void test_planner() {
  std::vector<TensorSpec> specs;
  std::vector<int> order;
  for (int i = 0; i < 40; ++i) {
    TensorSpec s;
    s.numel = 17 + 131 * i;
    s.elem_size = (i % 3 == 0) ? 2 : 4;
    s.dtype = i % 3 == 0 ? 1 : 0;
    specs.push_back(s);
    order.push_back(39 - i);
  }
  BucketPlan p = plan_buckets(specs, order, 8192, 256);
  for (int i = 0; i < 40; ++i) CHECK(p.tensor_bucket[i] >= 0);
  Controller c(p.tensor_bucket, (int)p.members.size(), 1);
  std::vector<int> released;
  for (int idx : order)
    for (int b : c.mark_ready(idx)) released.push_back(b);
  CHECK((int)released.size() == (int)p.members.size());
  for (size_t i = 0; i < released.size(); ++i) CHECK(released[i] == (int)i);
}

static void test_store_concurrency() {
  StoreServer srv("127.0.0.1", 0);
  const int kThreads = 8, kOps = 200;
  std::vector<std::thread> th;
  std::atomic<int> failures{0};
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      StoreClient c("127.0.0.1", srv.port(), 10.0);
      for (int i = 0; i < kOps; ++i) {
        c.add("counter", 1);
        c.set("k/" + std::to_string(t) + "/" + std::to_string(i), std::string(i % 50, 'x'));
        // every thread waits for the key written by its neighbour (parked GETs)
        const std::string want = "k/" + std::to_string((t + 1) % kThreads) + "/" + std::to_string(i);
        std::string v;
        if (!c.try_get(want, 10.0, &v) || v.size() != (size_t)(i % 50)) failures++;
      }
    });
  }
  for (auto& x : th) x.join();
  CHECK(failures.load() == 0);
  StoreClient c("127.0.0.1", srv.port(), 10.0);
  CHECK(c.add("counter", 0) == kThreads * kOps);
  CHECK(c.compare_set("cas", "", "a") == "a");
  CHECK(c.compare_set("cas", "b", "c") == "a");
  CHECK(!c.wait({"never"}, 0.02));
  srv.stop();
}

static void test_negotiator_threads() {
  StoreServer srv("127.0.0.1", 0);
  const int W = 4, N = 60;
  std::vector<std::unique_ptr<Negotiator>> negs;
  for (int r = 0; r < W; ++r)
    negs.emplace_back(new Negotiator("127.0.0.1", srv.port(), r, W, "st", 0.001, 0.0, 0.0));
  std::vector<std::vector<std::string>> got(W);
  std::vector<std::thread> th;
  for (int r = 0; r < W; ++r) {
    th.emplace_back([&, r] {
      std::vector<int> order(N);
      for (int i = 0; i < N; ++i) order[i] = i;
      std::mt19937 rng(1234 + r);
      std::shuffle(order.begin(), order.end(), rng);
      for (int i : order) negs[r]->submit("t" + std::to_string(i % 20), "sig");  // names reused 3x
      while ((int)got[r].size() < N)
        for (auto& x : negs[r]->wait(0.05)) got[r].push_back(x.name + "#" + std::to_string(x.generation));
    });
  }
  for (auto& x : th) x.join();
  for (int r = 1; r < W; ++r) CHECK(got[r] == got[0]);
  for (auto& n : negs) n->stop();
  srv.stop();
}

static void test_timeline_and_stall(const char* dir) {
  std::string path = std::string(dir) + "/selftest_timeline.json";
  {
    Timeline tl(path, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
      th.emplace_back([&, t] {
        for (int i = 0; i < 200; ++i) {
          tl.begin("op", "cat", t);
          tl.end("op", "cat", t);
        }
      });
    for (auto& x : th) x.join();
    tl.close();
    CHECK(tl.events_written() >= 1600);
  }
  StallInspector si(0.01, 0.0, 0.005, 0);
  si.set_hard_abort(false);
  si.start();
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&] {
      for (int i = 0; i < 100; ++i) si.complete(si.submit("x"));
    });
  const int64_t lonely = si.submit("lonely");
  for (auto& x : th) x.join();
  std::this_thread::sleep_for(std::chrono::milliseconds(60));
  CHECK(si.warnings_emitted() >= 1);
  si.complete(lonely);
  si.stop();
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  test_planner();
  test_store_concurrency();
  test_negotiator_threads();
  test_timeline_and_stall(dir);
  std::printf("runtime selftest ok\n");
  return 0;
}
