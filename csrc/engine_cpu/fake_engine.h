// In-process fake backend of the bucket engine (see fake_engine.cpp).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "comm/engine.h"

namespace hcb {
namespace fake {

uint16_t f32_to_bf16(float f);
float bf16_to_f32(uint16_t h);
uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);
float wire_round(float v, comm::Wire w);

struct RunConfig {
  int world = 2;
  comm::Wire wire = comm::Wire::F32;
  bool average = false;
  int64_t threshold_bytes = 128ll << 20;
  int stall_rank = -1;       // this rank's comm thread sleeps before bucket `stall_seq`
  int64_t stall_seq = -1;
  int stall_ms = 0;
  double warn_s = 0.0;       // > 0: run a watchdog per rank with this warn threshold
  // graph-replay emulation (the default multi-GPU path): the cycles are "captured" once (bucket
  // plan, no watch cycles), then replayed `replay_steps` times with no engine call per bucket;
  // with `heartbeat` each replay is followed by step_mark() -- the only thing the watchdog sees
  int replay_steps = 0;
  bool heartbeat = true;
  int stall_step = -1;       // replay mode: stall_rank's comm thread sleeps stall_ms in this step
};

struct Warning {
  int rank;
  int64_t cycle, last_seq;
  double waited_s;
};

// The collective rendezvous shared by all emulated ranks (keyed by the bucket sequence number,
// so a rank that issued a different schedule shows up as a size mismatch or a hang).
class FakeFabric {
 public:
  explicit FakeFabric(int world) : world_(world) {}
  void allreduce(int rank, int64_t seq, float* data, int64_t n, comm::Wire w, bool avg);
  void abort();
  int64_t mismatches() const { return mismatches_.load(); }

 private:
  struct Slot {
    int64_t n = -1;
    std::map<int, float*> ptrs;
    bool done = false;
    int departed = 0;
  };
  int world_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int64_t, Slot> slots_;
  std::atomic<int64_t> mismatches_{0};
  std::atomic<bool> aborted_{false};
};

// One emulated rank: the engine, its comm "stream" (an in-order worker thread) and watchdog.
class FakeRank final : public comm::Transport {
 public:
  FakeRank(int rank, FakeFabric* fab, const RunConfig& cfg);
  ~FakeRank() override;
  std::vector<comm::Bucket> submit(float* flat, int64_t numel, const std::vector<int64_t>& ranges, comm::Wire w,
                                   bool avg, int64_t threshold, bool do_join);
  // graph-replay emulation: enqueue a captured bucket schedule again (no watch cycle), and the
  // per-step heartbeat (one watch cycle completed behind the step's buckets)
  void replay(float* flat, const std::vector<comm::Bucket>& plan, comm::Wire w, bool avg, int step);
  void step_mark();
  void drain();
  std::vector<comm::Bucket> log() {
    std::lock_guard<std::mutex> lk(wmu_);
    return log_;
  }
  std::vector<Warning> warnings() {
    std::lock_guard<std::mutex> lk(wmu_);
    return warnings_;
  }
  int64_t cycles() const { return last_cycle_; }

  // Transport
  void fork() override {}
  void reduce_bucket(float* flat, const comm::Bucket& b, comm::Wire w, bool avg) override;
  void join() override { drain(); }
  void mark_cycle_end(int64_t cycle) override;

 private:
  void push(std::function<void()> op);
  void loop();
  void watch_loop();

  int rank_;
  FakeFabric* fab_;
  RunConfig cfg_;
  comm::BucketEngine engine_;
  comm::StallWatch watch_;
  std::mutex qmu_, wmu_;
  std::condition_variable qcv_;
  std::deque<std::function<void()>> q_;
  int pending_ = 0;
  bool stop_ = false;
  std::atomic<bool> stop_watch_{false};
  std::thread worker_, watchdog_;
  std::vector<comm::Bucket> log_;
  std::vector<Warning> warnings_;
  int64_t last_cycle_ = 0;
};

struct RunResult {
  std::vector<std::vector<float>> buffers;         // final buffer of every rank
  std::vector<std::vector<comm::Bucket>> buckets;  // buckets every rank issued, in order
  std::vector<Warning> warnings;
  std::vector<int64_t> cycles;
  int64_t size_mismatches = 0;
};

// Run `cycles` (each a flat list of (offset, length) pairs) on `cfg.world` emulated ranks whose
// buffers start as `init[r]`. Every cycle but the last uses the overlap (no-join) form.
RunResult run(const RunConfig& cfg, const std::vector<std::vector<float>>& init,
              const std::vector<std::vector<int64_t>>& cycles);

}  // namespace fake
}  // namespace hcb
