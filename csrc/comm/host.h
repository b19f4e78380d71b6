// Host-side bookkeeping of the communication runtime (csrc/comm/comm.cpp), kept free of HIP,
// RCCL and torch types so that it is compiled, unchanged, into the GPU library AND into the
// sanitizer stress driver (tools/sanitize/comm_host_stress.cpp, AddressSanitizer + UBSan and
// ThreadSanitizer; SURVEY.md §5 "Race detection / sanitizers"):
//   * HandleTable   -- the process-wide handle -> object maps (communicators, xGMI regions);
//   * EventPool     -- recycling of timing events (HOROVOD_TIMELINE records);
//   * Timeline      -- pending PACK / ALLREDUCE / UNPACK records and their Chrome-trace JSON;
//   * scratch_bytes -- growth rule of the compression wire buffer;
//   * WatchState    -- the per-cycle / per-step heartbeat bookkeeping around StallWatch
//                      (engine.h) that the caller's thread and the watchdog thread share;
//   * XgmiBook      -- rank / capacity / peer-mapping checks of the one-shot xGMI allreduce.
// The device side (events, streams) enters only through the functors the callers pass in.
#pragma once
#include <chrono>
#include <deque>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <ostream>
#include <string>
#include <utility>
#include <vector>

#include "comm/engine.h"

namespace hcb {
namespace comm {

// Thread-safe owning map from int64 handles (never reused, start at 1) to objects.
template <class T>
class HandleTable {
 public:
  int64_t add(std::unique_ptr<T> p) {
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t h = next_++;
    m_[h] = std::move(p);
    return h;
  }
  // nullptr for an unknown (or already destroyed) handle
  T* get(int64_t h) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(h);
    return it == m_.end() ? nullptr : it->second.get();
  }
  // removes and returns the object (empty for an unknown handle): the caller tears it down
  // outside the table lock
  std::unique_ptr<T> take(int64_t h) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(h);
    if (it == m_.end()) return nullptr;
    std::unique_ptr<T> p = std::move(it->second);
    m_.erase(it);
    return p;
  }
  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return m_.size();
  }

 private:
  std::mutex mu_;
  std::map<int64_t, std::unique_ptr<T>> m_;
  int64_t next_ = 1;
};

// Free list of device events; `create` makes a new one when the list is empty.
template <class Ev>
class EventPool {
 public:
  template <class Create>
  Ev get(Create&& create) {
    if (!free_.empty()) {
      Ev e = free_.back();
      free_.pop_back();
      return e;
    }
    ++created_;
    return create();
  }
  void put(Ev e) { free_.push_back(e); }
  template <class Destroy>
  void drain(Destroy&& destroy) {
    for (Ev e : free_) destroy(e);
    free_.clear();
  }
  size_t free_count() const { return free_.size(); }
  int64_t created() const { return created_; }

 private:
  std::vector<Ev> free_;
  int64_t created_ = 0;
};

template <class Ev>
struct TimelineRec {
  std::string name;
  int64_t bucket = 0;
  int64_t bytes = 0;
  Ev b{}, e{};
};

// HOROVOD_TIMELINE: intervals between two events per bucket, written as Chrome-trace "X"
// records once their end event has completed. Events go back to the pool when written (or
// dropped, with no timeline file open).
template <class Ev>
class Timeline {
 public:
  void open(std::ostream* out, int pid) {
    out_ = out;
    pid_ = pid;
    *out_ << "[\n";
  }
  bool is_open() const { return out_ != nullptr; }
  void record(TimelineRec<Ev> r) { pending_.push_back(std::move(r)); }
  size_t pending() const { return pending_.size(); }
  int64_t written() const { return written_; }

  // ready(e): non-blocking completion query; wait(e): block until complete; ms(e): milliseconds
  // of e since the timeline's base event. Without block, records whose end is not ready stay
  // pending (in order).
  template <class Ready, class Wait, class Ms>
  void flush(bool block, EventPool<Ev>& pool, Ready&& ready, Wait&& wait, Ms&& ms) {
    if (out_ == nullptr) {
      for (auto& r : pending_) {
        pool.put(r.b);
        pool.put(r.e);
      }
      pending_.clear();
      return;
    }
    std::vector<TimelineRec<Ev>> keep;
    for (auto& r : pending_) {
      if (!block && !ready(r.e)) {
        keep.push_back(r);
        continue;
      }
      wait(r.e);
      const double t0 = ms(r.b), t1 = ms(r.e);
      if (!first_) *out_ << ",\n";
      first_ = false;
      *out_ << "{\"name\":\"" << r.name << "\",\"ph\":\"X\",\"pid\":" << pid_ << ",\"tid\":" << r.bucket
            << ",\"ts\":" << t0 * 1000.0 << ",\"dur\":" << (t1 - t0) * 1000.0 << ",\"args\":{\"bytes\":" << r.bytes
            << ",\"bucket\":" << r.bucket << "}}";
      ++written_;
      pool.put(r.b);
      pool.put(r.e);
    }
    pending_.swap(keep);
    out_->flush();
  }
  void close() {
    if (out_ != nullptr) *out_ << "\n]\n";
    out_ = nullptr;
  }

 private:
  std::vector<TimelineRec<Ev>> pending_;
  std::ostream* out_ = nullptr;
  int pid_ = 0;
  bool first_ = true;
  int64_t written_ = 0;
};

// Compression wire buffer: bytes needed for a flat buffer of `numel` fp32 gradients shipped as
// `w`, or 0 when the current allocation `have` already suffices (grow-only: the allocation is
// reused by every later reduction, including graph-captured ones).
inline size_t scratch_bytes(size_t have, int64_t numel, Wire w) {
  if (w == Wire::F32 || numel <= 0) return 0;
  const size_t need = (size_t)numel * (size_t)wire_bytes(w);
  return need > have ? need : 0;
}

// Heartbeat bookkeeping shared by the caller's thread (eager reductions, step marks) and the
// watchdog thread. Every member function is called with the owner's mutex held; `done(ev)` is
// a non-blocking completion query of the single watch event.
struct WatchState {
  using clock = std::chrono::steady_clock;
  StallWatch watch;
  int64_t cycle = 0;         // the newest enqueued cycle
  int64_t first_mark = -1;   // first cycle enqueued by a step mark (graph-replayed steps)
  int64_t marks = 0;         // step marks seen
  clock::time_point last_call = clock::now();
  // every enqueued cycle with the token of the event recorded behind it, oldest first: each
  // cycle has an event of its own, so a caller that runs several steps ahead of the device (graph
  // replays never sync) still sees every one of them complete -- one re-recorded event would be
  // overwritten before it completed and the watchdog would report a stall of a healthy run
  std::deque<std::pair<int64_t, int64_t>> pending;

  // complete, oldest first, every pending cycle whose event has finished (done(token): a
  // non-blocking query); release(token) hands the event back to the owner's pool
  template <class Done, class Release>
  void retire(Done&& done, Release&& release) {
    while (!pending.empty() && done(pending.front().second)) {
      watch.complete(pending.front().first);
      release(pending.front().second);
      pending.pop_front();
    }
  }
  // the caller enters (a reduction or a step mark): note the time, retire finished cycles
  template <class Done, class Release>
  void enter(Done&& done, Release&& release) {
    last_call = clock::now();
    retire(done, release);
  }
  // after an event (token) was recorded behind the new work: one more cycle to watch
  int64_t enqueue(int64_t last_bucket, bool step_mark, int64_t token) {
    cycle = watch.enqueue(last_bucket);
    pending.emplace_back(cycle, token);
    if (step_mark) {
      ++marks;
      if (first_mark < 0) first_mark = cycle;
    }
    return cycle;
  }
  // the watchdog thread, when the caller has been quiet for > quiet_s (blocked on a hung
  // collective or idle): it may query the events itself
  template <class Done, class Release>
  void poll_quiet(clock::time_point now, double quiet_s, Done&& done, Release&& release) {
    if (!pending.empty() && std::chrono::duration<double>(now - last_call).count() > quiet_s) retire(done, release);
  }
  bool is_graph_cycle(int64_t c) const { return first_mark >= 0 && c >= first_mark; }
};

// One-shot xGMI allreduce bookkeeping (the device protocol is csrc/kernels/xgmi.hip).
struct XgmiBook {
  int rank = 0, world = 1;
  int64_t cap = 0;  // floats per slot
  std::vector<void*> peers;
  std::vector<bool> opened;

  // "" when (rank, world, cap) is a valid region request, else the reason
  static std::string check_create(int64_t rank, int64_t world, int64_t cap, int max_ranks) {
    if (world < 1 || world > max_ranks || rank < 0 || rank >= world)
      return "1.." + std::to_string(max_ranks) + " ranks, 0 <= rank < world";
    if (cap <= 0 || cap % 4 != 0) return "capacity must be a positive multiple of 4 floats";
    if (cap > (int64_t(1) << 35)) return "capacity above 2^35 floats (128 GiB per slot)";
    return "";
  }
  // bytes of one region: two slots of `cap` floats + 256 bytes of flags
  static size_t region_bytes(int64_t cap) { return (size_t)2 * (size_t)cap * 4 + 256; }
  void init(int r, int w, int64_t c, void* own) {
    rank = r;
    world = w;
    cap = c;
    peers.assign(w, nullptr);
    opened.assign(w, false);
    peers[r] = own;
  }
  void set_peer(int r, void* p) {
    peers.at(r) = p;
    opened.at(r) = true;
  }
  // "" when a reduction of `numel` floats may be launched, else the reason
  std::string check_reduce(int64_t numel) const {
    if (numel > cap) return std::to_string(numel) + " floats > capacity " + std::to_string(cap);
    for (int r = 0; r < world; ++r)
      if (peers[r] == nullptr) return "peer " + std::to_string(r) + " not opened";
    return "";
  }
};

}  // namespace comm
}  // namespace hcb
