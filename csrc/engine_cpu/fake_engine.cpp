// In-process fake backend for the gradient bucket engine (csrc/comm/engine.h): W ranks are
// emulated by threads, each with its own flat gradient buffer, BucketEngine, comm "stream"
// (a worker thread executing the enqueued bucket reductions strictly in order) and stall
// watchdog; a shared FakeFabric rendezvous performs the collectives (sum / average with the
// wire format's rounding: fp32, bf16 or IEEE fp16).
//
// It runs the SAME engine code as the RCCL build (bucket planning, sequence numbering, cycle
// accounting, StallWatch) with no GPU, so the CPU test suite can check bucket ordering across
// ranks, the HOROVOD_FUSION_THRESHOLD split, compression numerics and the stall watchdog
// (SURVEY.md §7.5 "fake in-process backend"). Exposed to Python with pybind11
// (tests/test_engine_fake.py); tools/sanitize/engine_stress.cpp drives it under ASan/UBSan
// and TSan.
#include "fake_engine.h"

#include <cmath>
#include <cstring>

namespace hcb {
namespace fake {

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
// IEEE binary16, round to nearest even, overflow -> inf (what a hardware cvt does)
uint16_t f32_to_f16(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7fffffffu;
  if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u);
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // >= 65520 rounds to inf
  if (ax < 0x38800000u) {                                     // subnormal half (or zero)
    if (ax < 0x33000000u) return (uint16_t)sign;              // < 2^-25: rounds to 0
    const uint32_t m = (ax & 0x7fffffu) | 0x800000u;
    const int e = (int)(ax >> 23);
    const int shift = 126 - e;  // the result is in units of 2^-24: m * 2^(e - 150) / 2^-24
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (r & 1u))) ++r;
    return (uint16_t)(sign | r);
  }
  uint32_t r = ((ax >> 13) - (112u << 10));
  const uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) ++r;
  return (uint16_t)(sign | r);
}
float f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
  float f;
  if (e == 0) {
    f = std::ldexp((float)m, -24);
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u |= sign;
    std::memcpy(&f, &u, 4);
    return f;
  }
  uint32_t u = e == 31 ? (sign | 0x7f800000u | (m << 13)) : (sign | ((e + 112) << 23) | (m << 13));
  std::memcpy(&f, &u, 4);
  return f;
}
float wire_round(float v, comm::Wire w) {
  switch (w) {
    case comm::Wire::BF16: return bf16_to_f32(f32_to_bf16(v));
    case comm::Wire::F16: return f16_to_f32(f32_to_f16(v));
    default: return v;
  }
}

// ------------------------------------------------------------------------------ fabric
void FakeFabric::allreduce(int rank, int64_t seq, float* data, int64_t n, comm::Wire w, bool avg) {
  std::unique_lock<std::mutex> lk(mu_);
  Slot& s = slots_[seq];
  if (s.n < 0) s.n = n;
  if (s.n != n) {
    mismatches_.fetch_add(1);
    s.n = std::max(s.n, n);
  }
  s.ptrs[rank] = data;
  if ((int)s.ptrs.size() == world_) {
    // last arriver: every rank's packed contribution is rounded to the wire format, summed in
    // rank order (deterministic), averaged, and rounded again as the wire result
    std::vector<float> acc(n, 0.f);
    for (int r = 0; r < world_; ++r) {
      const float* p = s.ptrs[r];
      for (int64_t i = 0; i < n; ++i) acc[i] += wire_round(p[i], w);
    }
    for (int64_t i = 0; i < n; ++i) {
      float v = acc[i];
      if (avg) v /= (float)world_;
      acc[i] = wire_round(v, w);
    }
    for (int r = 0; r < world_; ++r) std::memcpy(s.ptrs[r], acc.data(), n * sizeof(float));
    s.done = true;
    cv_.notify_all();
  } else {
    cv_.wait(lk, [&] { return s.done || aborted_.load(); });
  }
  if (++s.departed == world_) slots_.erase(seq);
}

void FakeFabric::abort() {
  std::lock_guard<std::mutex> lk(mu_);
  aborted_ = true;
  cv_.notify_all();
}

// ------------------------------------------------------------------------------ rank
FakeRank::FakeRank(int rank, FakeFabric* fab, const RunConfig& cfg)
    : rank_(rank), fab_(fab), cfg_(cfg), engine_(this) {
  watch_.configure(cfg.warn_s, 0.0);
  worker_ = std::thread([this] { loop(); });
  if (cfg.warn_s > 0) watchdog_ = std::thread([this] { watch_loop(); });
}

FakeRank::~FakeRank() {
  {
    std::lock_guard<std::mutex> lk(qmu_);
    stop_ = true;
  }
  qcv_.notify_all();
  if (worker_.joinable()) worker_.join();
  stop_watch_ = true;
  if (watchdog_.joinable()) watchdog_.join();
}

void FakeRank::push(std::function<void()> op) {
  {
    std::lock_guard<std::mutex> lk(qmu_);
    q_.push_back(std::move(op));
    ++pending_;
  }
  qcv_.notify_all();
}

void FakeRank::loop() {
  for (;;) {
    std::function<void()> op;
    {
      std::unique_lock<std::mutex> lk(qmu_);
      qcv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      op = std::move(q_.front());
      q_.pop_front();
    }
    op();
    {
      std::lock_guard<std::mutex> lk(qmu_);
      --pending_;
    }
    qcv_.notify_all();
  }
}

void FakeRank::drain() {
  std::unique_lock<std::mutex> lk(qmu_);
  qcv_.wait(lk, [&] { return pending_ == 0; });
}

void FakeRank::watch_loop() {
  using comm::StallWatch;
  while (!stop_watch_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    double waited = 0;
    StallWatch::Action a = watch_.evaluate(StallWatch::clock::now(), &waited);
    if (a == StallWatch::kWarn) {
      std::lock_guard<std::mutex> lk(wmu_);
      warnings_.push_back({rank_, watch_.completed() + 1, watch_.last_seq(), waited});
    }
  }
}

void FakeRank::reduce_bucket(float* flat, const comm::Bucket& b, comm::Wire w, bool avg) {
  {
    std::lock_guard<std::mutex> lk(wmu_);
    log_.push_back(b);
  }
  const int64_t seq = b.seq;
  const comm::Bucket bb = b;
  push([this, flat, bb, w, avg, seq] {
    if (rank_ == cfg_.stall_rank && seq == cfg_.stall_seq && cfg_.stall_ms > 0)
      std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.stall_ms));
    fab_->allreduce(rank_, seq, flat + bb.off, bb.len, w, avg);
  });
}

void FakeRank::mark_cycle_end(int64_t cycle) {
  last_cycle_ = cycle;
  const int64_t last_seq = engine_.next_seq() - 1;
  watch_.enqueue(last_seq);
  push([this, cycle] { watch_.complete(cycle); });
}

void FakeRank::replay(float* flat, const std::vector<comm::Bucket>& plan, comm::Wire w, bool avg, int step) {
  const bool stall = rank_ == cfg_.stall_rank && step == cfg_.stall_step && cfg_.stall_ms > 0;
  for (size_t i = 0; i < plan.size(); ++i) {
    const comm::Bucket b = plan[i];
    // a fresh rendezvous key per replay (the fabric slot of step k is freed once all departed)
    const int64_t key = (int64_t)step * 1000000 + b.seq;
    const bool sleep = stall && i == 0;
    push([this, flat, b, w, avg, key, sleep] {
      if (sleep) std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.stall_ms));
      fab_->allreduce(rank_, key, flat + b.off, b.len, w, avg);
    });
  }
}

void FakeRank::step_mark() {
  const int64_t cycle = watch_.enqueue(engine_.next_seq() - 1);
  last_cycle_ = cycle;
  push([this, cycle] { watch_.complete(cycle); });
}

std::vector<comm::Bucket> FakeRank::submit(float* flat, int64_t numel, const std::vector<int64_t>& ranges,
                                           comm::Wire w, bool avg, int64_t threshold, bool do_join) {
  return engine_.submit(flat, numel, ranges.data(), (int64_t)ranges.size() / 2, w, avg, threshold, do_join);
}

// ------------------------------------------------------------------------------ driver
RunResult run(const RunConfig& cfg, const std::vector<std::vector<float>>& init,
              const std::vector<std::vector<int64_t>>& cycles) {
  const int W = cfg.world;
  RunResult res;
  res.buffers = init;
  FakeFabric fab(W);
  std::vector<std::unique_ptr<FakeRank>> ranks;
  for (int r = 0; r < W; ++r) ranks.emplace_back(new FakeRank(r, &fab, cfg));
  std::vector<std::thread> mains;
  std::vector<std::string> errors(W);
  for (int r = 0; r < W; ++r) {
    mains.emplace_back([&, r] {
      try {
        float* flat = res.buffers[r].data();
        const int64_t numel = (int64_t)res.buffers[r].size();
        if (cfg.replay_steps > 0) {
          // capture: the step's bucket schedule, planned exactly as submit() plans it
          std::vector<comm::Bucket> plan;
          for (const auto& c : cycles) {
            auto bs = comm::plan_buckets(c.data(), (int64_t)c.size() / 2,
                                         comm::bucket_elems_for(cfg.threshold_bytes, cfg.wire));
            for (auto& b : bs) {
              if (b.off < 0 || b.off + b.len > numel) throw std::out_of_range("bucket out of range");
              b.seq = (int64_t)plan.size();
              plan.push_back(b);
            }
          }
          for (int s = 0; s < cfg.replay_steps; ++s) {
            ranks[r]->replay(flat, plan, cfg.wire, cfg.average, s);
            if (cfg.heartbeat) ranks[r]->step_mark();
          }
        } else {
          for (size_t c = 0; c < cycles.size(); ++c) {
            const bool last = c + 1 == cycles.size();
            ranks[r]->submit(flat, numel, cycles[c], cfg.wire, cfg.average, cfg.threshold_bytes, last);
          }
        }
        ranks[r]->drain();
      } catch (const std::exception& e) {
        errors[r] = e.what();
        fab.abort();
      }
    });
  }
  for (auto& t : mains) t.join();
  for (int r = 0; r < W; ++r) {
    if (!errors[r].empty()) throw std::runtime_error("rank " + std::to_string(r) + ": " + errors[r]);
    res.buckets.push_back(ranks[r]->log());
    for (auto& wv : ranks[r]->warnings()) res.warnings.push_back(wv);
    res.cycles.push_back(ranks[r]->cycles());
  }
  res.size_mismatches = fab.mismatches();
  ranks.clear();
  return res;
}

}  // namespace fake
}  // namespace hcb
