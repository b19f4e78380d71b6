// Sanitizer stress driver for the HIP-free host bookkeeping of the communication runtime
// (csrc/comm/host.h, used by csrc/comm/comm.cpp): handle tables under concurrent create /
// lookup / destroy, event recycling through the timeline, the watch-state protocol between a
// submitting thread, a fake device and the watchdog thread (healthy progress, then a stall that
// must warn and abort), the compression-scratch growth rule and the xGMI bookkeeping checks.
// Built with -fsanitize=address,undefined and with -fsanitize=thread by
// tools/sanitize/run_engine_sanitizers.sh; exits non-zero on any failed check.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "comm/host.h"

using namespace hcb::comm;
using clk = std::chrono::steady_clock;

#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "comm_host_stress: CHECK failed: %s (line %d)\n", #c, __LINE__); \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

// a fake device event: completes when the fake device reaches its sequence number
struct FakeDevice {
  std::atomic<int64_t> reached{0};
  std::atomic<bool> stalled{false};
};
struct FakeEv {
  int64_t seq = 0;
  double t_ms = 0;
};

static void handle_tables() {
  struct Obj {
    std::vector<int> payload = std::vector<int>(64, 7);
  };
  HandleTable<Obj> t;
  std::atomic<int64_t> bad{0};
  std::vector<std::thread> th;
  for (int w = 0; w < 8; ++w)
    th.emplace_back([&] {
      std::vector<int64_t> mine;
      for (int i = 0; i < 3000; ++i) {
        mine.push_back(t.add(std::make_unique<Obj>()));
        Obj* o = t.get(mine.back());
        if (!o || o->payload[63] != 7) bad++;
        if (i % 3 == 2) {
          auto p = t.take(mine.front());
          if (!p) bad++;
          if (t.get(mine.front()) != nullptr) bad++;
          mine.erase(mine.begin());
        }
      }
      for (int64_t h : mine) t.take(h);
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0);
  CHECK(t.size() == 0);
  CHECK(t.get(1) == nullptr && !t.take(12345));
}

static void timeline_and_pool() {
  std::vector<std::unique_ptr<FakeEv>> owned;
  EventPool<FakeEv*> pool;
  auto create = [&] {
    owned.push_back(std::make_unique<FakeEv>());
    return owned.back().get();
  };
  std::ostringstream out;
  Timeline<FakeEv*> tl;
  tl.open(&out, 3);
  FakeDevice dev;
  int64_t seq = 0;
  std::atomic<bool> stop{false};
  std::thread device([&] {  // completes events in order, a little behind the submitter
    while (!stop.load()) {
      dev.reached.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  });
  auto ready = [&](FakeEv* e) { return dev.reached.load() >= e->seq; };
  auto wait = [&](FakeEv* e) {
    while (dev.reached.load() < e->seq) std::this_thread::yield();
  };
  auto ms = [](FakeEv* e) { return e->t_ms; };
  const int N = 2000;
  for (int i = 0; i < N; ++i) {
    FakeEv* b = pool.get(create);
    FakeEv* e = pool.get(create);
    b->seq = ++seq;
    b->t_ms = 0.01 * (double)seq;
    e->seq = ++seq;
    e->t_ms = 0.01 * (double)seq;
    tl.record({i % 2 ? "ALLREDUCE" : "PACK_ALLREDUCE_UNPACK", i, 4096 * (int64_t)i, b, e});
    if (i % 16 == 15) tl.flush(false, pool, ready, wait, ms);
  }
  tl.flush(true, pool, ready, wait, ms);
  stop = true;
  device.join();
  CHECK(tl.pending() == 0 && tl.written() == N);
  CHECK((int64_t)pool.free_count() == pool.created());  // every event came back
  CHECK(pool.created() < 2 * N);                           // and was reused
  tl.close();
  const std::string s = out.str();
  size_t recs = 0;
  for (size_t p = s.find("\"ph\":\"X\""); p != std::string::npos; p = s.find("\"ph\":\"X\"", p + 1)) ++recs;
  CHECK(recs == (size_t)N);
  CHECK(s.rfind("[\n", 0) == 0 && s.size() > 3 && s.substr(s.size() - 3) == "\n]\n");
  // without a file the records are dropped and the events recycled
  Timeline<FakeEv*> off;
  FakeEv* b = pool.get(create);
  FakeEv* e = pool.get(create);
  off.record({"ALLREDUCE", 0, 4, b, e});
  const size_t before = pool.free_count();
  off.flush(false, pool, ready, wait, ms);
  CHECK(off.pending() == 0 && pool.free_count() == before + 2);
  int destroyed = 0;
  pool.drain([&](FakeEv*) { ++destroyed; });
  CHECK(destroyed == (int)pool.created() && pool.free_count() == 0);
}

// submitter (caller's thread) + fake device + watchdog, sharing one WatchState under a mutex; each
// enqueued cycle records its own fake event (the device sequence number it completes at)
static void watch_protocol() {
  WatchState ws;
  ws.watch.configure(0.25, 0.8);
  std::mutex mu;
  FakeDevice dev;
  std::vector<int64_t> ev_target;  // token -> device sequence (guarded by mu)
  std::vector<int64_t> ev_free;
  std::atomic<int64_t> dev_target{0};
  std::atomic<bool> stop{false}, warned{false}, aborted{false};
  auto done = [&](int64_t t) { return dev.reached.load() >= ev_target[t]; };
  auto release = [&](int64_t t) { ev_free.push_back(t); };
  auto record = [&](int64_t seq) {
    int64_t t;
    if (!ev_free.empty()) {
      t = ev_free.back();
      ev_free.pop_back();
      ev_target[t] = seq;
    } else {
      ev_target.push_back(seq);
      t = (int64_t)ev_target.size() - 1;
    }
    return t;
  };
  std::atomic<int> dev_delay_us{20};
  std::thread device([&] {
    while (!stop.load()) {
      if (!dev.stalled.load() && dev.reached.load() < dev_target.load()) dev.reached.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(dev_delay_us.load()));
    }
  });
  std::thread watchdog([&] {
    while (!stop.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      const auto now = clk::now();
      {
        std::lock_guard<std::mutex> lk(mu);
        ws.poll_quiet(now, 0.05, done, release);
      }
      double waited = 0;
      const StallWatch::Action a = ws.watch.evaluate(now, &waited);
      if (a == StallWatch::kWarn) warned = true;
      if (a == StallWatch::kAbort) aborted = true;
    }
  });
  // healthy phase: 400 cycles (eager reductions and step marks alternately)
  for (int i = 0; i < 400; ++i) {
    std::lock_guard<std::mutex> lk(mu);
    ws.enter(done, release);
    const int64_t t = dev_target.fetch_add(1) + 1;  // the work of this cycle
    ws.enqueue(i, i % 2 == 1, record(t));            // its own event recorded behind it
    if (i % 50 == 0) {
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  // drain: the watchdog completes the last cycles once the caller is quiet
  auto drain = [&] {
    const auto t0 = clk::now();
    while (ws.watch.completed() < ws.watch.enqueued() && clk::now() - t0 < std::chrono::seconds(5))
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
  };
  drain();
  CHECK(ws.watch.completed() == ws.watch.enqueued());
  CHECK(!warned.load() && !aborted.load());
  {
    std::lock_guard<std::mutex> lk(mu);
    CHECK(ws.marks == 200 && ws.first_mark == 2 && ws.is_graph_cycle(400) && !ws.is_graph_cycle(1));
    CHECK(ws.pending.empty() && ev_free.size() == ev_target.size());
  }
  // the caller runs far ahead of a slow device (graph replays never sync) for longer than the warn
  // threshold: the device keeps completing cycles, so no stall may be reported (with one
  // re-recorded event the earlier cycles were never seen completing)
  dev_delay_us = 2000;
  const auto ta = clk::now();
  for (int i = 0; clk::now() - ta < std::chrono::milliseconds(600); ++i) {
    {
      std::lock_guard<std::mutex> lk(mu);
      ws.enter(done, release);
      const int64_t t = dev_target.fetch_add(1) + 1;
      ws.enqueue(400 + i, true, record(t));
    }
    std::this_thread::sleep_for(std::chrono::microseconds(300));  // 6-7x faster than the device
  }
  CHECK(!warned.load() && !aborted.load());
  dev_delay_us = 20;
  drain();
  CHECK(ws.watch.completed() == ws.watch.enqueued());
  CHECK(!warned.load() && !aborted.load());
  // stall phase: the device stops; one more cycle must warn, then abort
  dev.stalled = true;
  {
    std::lock_guard<std::mutex> lk(mu);
    ws.enter(done, release);
    ws.enqueue(100000, true, record(dev_target.fetch_add(1) + 1));
  }
  const auto t1 = clk::now();
  while (!aborted.load() && clk::now() - t1 < std::chrono::seconds(5))
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  CHECK(warned.load() && aborted.load());
  stop = true;
  device.join();
  watchdog.join();
}

static void scratch_and_xgmi() {
  CHECK(scratch_bytes(0, 1000, Wire::F32) == 0);
  CHECK(scratch_bytes(0, 1000, Wire::BF16) == 2000);
  CHECK(scratch_bytes(2000, 1000, Wire::F16) == 0);
  CHECK(scratch_bytes(2000, 1001, Wire::F16) == 2002);
  CHECK(scratch_bytes(0, -5, Wire::BF16) == 0);
  CHECK(scratch_bytes(0, int64_t(25557032), Wire::BF16) == size_t(51114064));
  CHECK(XgmiBook::check_create(0, 8, 1 << 20, 8).empty());
  CHECK(!XgmiBook::check_create(8, 8, 1 << 20, 8).empty());
  CHECK(!XgmiBook::check_create(-1, 8, 1 << 20, 8).empty());
  CHECK(!XgmiBook::check_create(0, 9, 1 << 20, 8).empty());
  CHECK(!XgmiBook::check_create(0, 0, 1 << 20, 8).empty());
  CHECK(!XgmiBook::check_create(0, 2, 6, 8).empty());
  CHECK(!XgmiBook::check_create(0, 2, 0, 8).empty());
  CHECK(!XgmiBook::check_create(0, 2, INT64_MAX - 3, 8).empty());  // would overflow region_bytes
  CHECK(XgmiBook::region_bytes(1 << 20) == size_t(8u << 20) + 256);
  int own = 0, peer = 0;
  XgmiBook b;
  b.init(1, 3, 1024, &own);
  CHECK(!b.check_reduce(16).empty());  // peers 0 and 2 not opened
  b.set_peer(0, &peer);
  b.set_peer(2, &peer);
  CHECK(b.check_reduce(1024).empty());
  CHECK(!b.check_reduce(1025).empty());
  bool threw = false;
  try {
    b.set_peer(3, &peer);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  CHECK(threw);
}

int main() {
  handle_tables();
  timeline_and_pool();
  watch_protocol();
  scratch_and_xgmi();
  std::printf("comm_host_stress: ok\n");
  return 0;
}
