// Transport-independent core of the gradient bucket engine: bucket planning, the in-order
// enqueue of a reduction cycle, progress accounting and the stall-watchdog decision.
//
// The reference's Horovod core (SURVEY.md §2.2 "Horovod core", §5 "Failure detection";
// knobs at /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:105-106) packs ready
// tensors into a fusion buffer of at most HOROVOD_FUSION_THRESHOLD bytes, reduces each buffer
// with one MPI_Allreduce and warns (stall inspector) when ranks disagree for too long. Here:
//   * the fusion buffer IS the flat gradient storage, so a "bucket" is an (offset, length)
//     slice; every backward-segment range handed to the engine is cut into buckets of at most
//     the threshold (wire bytes) in a fixed order that is identical on every rank -- no
//     negotiation, because the schedule is static;
//   * a Transport enqueues the pack / collective / unpack of one bucket on its comm stream
//     (RCCL on a HIP stream in comm.cpp; an in-process threaded fabric in engine_cpu.cpp, the
//     fake backend the CPU tests drive);
//   * StallWatch turns (enqueued, completed, time) into warn / abort decisions, with the
//     stalled cycle and bucket named.
// No HIP, RCCL or torch types appear here, so the same code is compiled into the GPU
// library and into the CPU test library.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace hcb {
namespace comm {

enum class Wire : int { F32 = 0, BF16 = 1, F16 = 2 };

inline int wire_bytes(Wire w) { return w == Wire::F32 ? 4 : 2; }

struct Bucket {
  int64_t off = 0, len = 0;  // elements of the flat fp32 buffer
  int64_t seq = 0;           // position in the engine's lifetime schedule (same on every rank)
};

// Cut each (offset, length) range into pieces of at most max_elems elements, in order. A
// piece boundary is kept a multiple of `align` elements from the range start so that packed
// wire buffers stay 16-byte aligned. max_elems <= 0 means "no limit".
inline std::vector<Bucket> plan_buckets(const int64_t* ranges, int64_t nranges, int64_t max_elems,
                                        int64_t align = 64) {
  std::vector<Bucket> out;
  if (max_elems > 0) max_elems = std::max<int64_t>(align, max_elems / align * align);
  for (int64_t r = 0; r < nranges; ++r) {
    int64_t off = ranges[2 * r], len = ranges[2 * r + 1];
    if (len <= 0) continue;
    if (max_elems <= 0) {
      out.push_back({off, len, 0});
      continue;
    }
    // equal-sized pieces (no tiny tail): ceil(len / max) pieces of ~len / pieces each
    const int64_t pieces = (len + max_elems - 1) / max_elems;
    int64_t per = (len + pieces - 1) / pieces;
    per = std::min(max_elems, (per + align - 1) / align * align);
    for (int64_t s = 0; s < len; s += per) out.push_back({off + s, std::min(per, len - s), 0});
  }
  return out;
}

// Bytes of wire buffer a bucket's threshold allows.
inline int64_t bucket_elems_for(int64_t threshold_bytes, Wire w) {
  return threshold_bytes <= 0 ? 0 : std::max<int64_t>(1, threshold_bytes / wire_bytes(w));
}

// What a transport must provide. All calls enqueue work on the transport's comm stream,
// which runs the buckets strictly in enqueue order.
struct Transport {
  virtual ~Transport() = default;
  // comm stream waits for everything the caller's stream has enqueued so far
  virtual void fork() = 0;
  // reduce elements [off, off + len) of `flat` in place (sum, or average when avg), shipping
  // them over the wire as `w` (pack -> collective -> unpack when w != F32)
  virtual void reduce_bucket(float* flat, const Bucket& b, Wire w, bool avg) = 0;
  // caller's stream waits for the comm stream (join) -- or not, for the overlap form
  virtual void join() = 0;
  // mark the end of one engine cycle; `cycle` is monotonically increasing
  virtual void mark_cycle_end(int64_t cycle) = 0;
  // timeline hooks (optional)
  virtual void bucket_begin(const Bucket&) {}
  virtual void bucket_end(const Bucket&, Wire) {}
};

// Progress accounting + stall decision. enqueue() is called by the submitting thread after a
// cycle was enqueued; complete(c) by whoever observes that cycle c has finished (an event query
// on the GPU, the fake comm thread on the CPU). evaluate() is the watchdog's pure decision.
class StallWatch {
 public:
  using clock = std::chrono::steady_clock;
  enum Action { kIdle = 0, kProgress = 1, kWaiting = 2, kWarn = 3, kAbort = 4 };

  StallWatch(double warn_s = 60.0, double abort_s = 0.0) : warn_s_(warn_s), abort_s_(abort_s) {}
  void configure(double warn_s, double abort_s) {
    warn_s_ = warn_s;
    abort_s_ = abort_s;
  }

  int64_t enqueue(int64_t last_seq) {
    last_seq_.store(last_seq, std::memory_order_relaxed);
    return enq_.fetch_add(1, std::memory_order_acq_rel) + 1;
  }
  void complete(int64_t cycle) {
    int64_t d = done_.load(std::memory_order_acquire);
    while (cycle > d && !done_.compare_exchange_weak(d, cycle, std::memory_order_acq_rel)) {
    }
  }
  int64_t enqueued() const { return enq_.load(std::memory_order_acquire); }
  int64_t completed() const { return done_.load(std::memory_order_acquire); }
  int64_t last_seq() const { return last_seq_.load(std::memory_order_relaxed); }

  // One watchdog look at time `now`. Returns the action; `waited` is the time without progress.
  Action evaluate(clock::time_point now, double* waited = nullptr) {
    const int64_t d = completed(), e = enqueued();
    if (d >= e) {
      seen_ = d;
      since_ = now;
      warned_ = false;
      if (waited) *waited = 0;
      return kIdle;
    }
    if (d != seen_) {
      seen_ = d;
      since_ = now;
      warned_ = false;
      if (waited) *waited = 0;
      return kProgress;
    }
    const double w = std::chrono::duration<double>(now - since_).count();
    if (waited) *waited = w;
    if (abort_s_ > 0 && w > abort_s_) return kAbort;
    if (!warned_ && w > warn_s_) {
      warned_ = true;
      return kWarn;
    }
    return kWaiting;
  }
  double warn_s() const { return warn_s_; }
  double abort_s() const { return abort_s_; }

 private:
  std::atomic<int64_t> enq_{0}, done_{0}, last_seq_{-1};
  int64_t seen_ = -1;
  bool warned_ = false;
  clock::time_point since_ = clock::now();
  double warn_s_, abort_s_;
};

// The engine: one call = one cycle over the given ranges.
class BucketEngine {
 public:
  explicit BucketEngine(Transport* t) : t_(t) {}

  // Returns the buckets issued (with their lifetime sequence numbers).
  std::vector<Bucket> submit(float* flat, int64_t numel, const int64_t* ranges, int64_t nranges, Wire w, bool avg,
                             int64_t threshold_bytes, bool do_join) {
    std::vector<Bucket> bs = plan_buckets(ranges, nranges, bucket_elems_for(threshold_bytes, w));
    for (auto& b : bs) {
      if (b.off < 0 || b.off + b.len > numel) throw std::out_of_range("hcb bucket engine: bucket out of range");
      b.seq = next_seq_++;
    }
    t_->fork();
    for (const auto& b : bs) {
      t_->bucket_begin(b);
      t_->reduce_bucket(flat, b, w, avg);
      t_->bucket_end(b, w);
    }
    if (do_join) t_->join();
    ++cycle_;
    t_->mark_cycle_end(cycle_);
    return bs;
  }
  int64_t cycle() const { return cycle_; }
  int64_t next_seq() const { return next_seq_; }

 private:
  Transport* t_;
  int64_t cycle_ = 0, next_seq_ = 0;
};

}  // namespace comm
}  // namespace hcb
