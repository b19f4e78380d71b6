// Native data-parallel communication runtime for MI355X: RCCL communicator + bucketed
// gradient allreduce engine on a side HIP stream + Chrome-trace timeline + stall watchdog.
//
// This is the MI355X replacement for the Horovod C++ core the reference drives
// (background thread, tensor-fusion buffer, MPI_Allreduce, HOROVOD_TIMELINE, stall
// inspector; SURVEY.md §2.2 "Horovod core", §2.3, §5; reference knobs at
// /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:105-106). Design:
//   * no negotiation: every rank runs the same static bucket schedule over ONE flat
//     gradient buffer (the fusion buffer IS the gradient storage), so a "cycle" is just
//     a sequence of ncclAllReduce calls;
//   * the communicator is created from an ncclUniqueId exchanged through the
//     torch.distributed TCP store (no MPI);
//   * collectives run on a dedicated comm stream forked from / joined back to the
//     caller's stream with HIP events (capturable into a HIP graph);
//   * optional bf16/fp16 compression: pack kernel (scale+cast) -> allreduce -> unpack,
//     all on the comm stream;
//   * timeline: per-bucket PACK / ALLREDUCE / UNPACK intervals measured with HIP events
//     and written as Chrome trace JSON (HOROVOD_TIMELINE);
//   * watchdog thread: warns when a launched reduction has not completed within
//     HOROVOD_STALL_CHECK_TIME_SECONDS, polls ncclCommGetAsyncError, optionally aborts
//     the communicator (HCB_STALL_ABORT_SECONDS) so a dead rank cannot hang the job.
//     Eager reductions are watched per call; on the default multi-GPU path the collectives
//     live inside the replayed step graph (no host call per reduction), so the trainer calls
//     step_mark() after every replay: one watch cycle per step, completed by an event recorded
//     on the caller's stream behind the graph (whose comm branch joins before its end).
#include <torch/library.h>
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <ATen/ops/zeros.h>
#include <c10/hip/HIPStream.h>
#include <c10/util/Exception.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "comm/engine.h"
#include "comm/host.h"
#include "kernels/kernels.h"

using at::Tensor;

#define HCB_HIP(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    TORCH_CHECK(e_ == hipSuccess, "hcb_comm: ", #x, " failed: ", hipGetErrorString(e_)); \
  } while (0)
#define HCB_NCCL(x)                                                                     \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    TORCH_CHECK(r_ == ncclSuccess, "hcb_comm: ", #x, " failed: ", ncclGetErrorString(r_)); \
  } while (0)

namespace {

double env_double(const char* name, double dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return std::atof(v);
}

ncclDataType_t nccl_type(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "hcb_comm: unsupported dtype ", t.scalar_type());
  }
}

struct Comm {
  // process exit without destroy() (static destruction of g_comms): stop and join the
  // watchdog thread -- a joinable std::thread would std::terminate -- and touch nothing else
  // (HIP / RCCL may already be torn down)
  ~Comm() {
    stop = true;
    cv.notify_all();
    if (wd.joinable()) wd.join();
  }
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  hipStream_t stream = nullptr;  // comm stream
  hipEvent_t fork_ev = nullptr, join_ev = nullptr, base_ev = nullptr;
  // compression scratch (grown on demand, owned by the engine)
  void* cbuf = nullptr;
  size_t cbuf_bytes = 0;
  // timeline (HIP-free bookkeeping in comm/host.h)
  std::string timeline_path;
  std::ofstream tl_file;
  hcb::comm::Timeline<hipEvent_t> timeline;
  hcb::comm::EventPool<hipEvent_t> events;
  int64_t cycle = 0;
  int64_t buckets_issued = 0;  // lifetime count of bucket collectives
  // watchdog
  std::thread wd;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<bool> stop{false};
  // Progress counters for the watchdog. The watchdog thread never calls into HIP or RCCL
  // while the job is healthy: with a second host thread querying the comm stream's events
  // (or host callbacks on that stream) the training step was corrupted intermittently on
  // MI355X (tools/dp_variants.sh). Instead the CALLER's thread, at each new reduction,
  // polls the previous cycle's dedicated watch event and advances `done`; the watchdog
  // thread only compares `done` with `enq` and the clock. Only when the caller has been
  // quiet for > 1 s (blocked on a hung collective, or idle) does the watchdog query the
  // watch event itself, under `mu`, which every enqueue also holds.
  hcb::comm::WatchState ws;  // guarded by mu (ws.watch's counters are atomics)
  std::unique_ptr<hcb::comm::Transport> transport;  // RcclTransport, created on first use
  std::unique_ptr<hcb::comm::BucketEngine> engine;  // lifetime bucket numbering
  int64_t fusion_bytes = 128ll << 20;  // HOROVOD_FUSION_THRESHOLD
  // debug (HCB_COMM_DEBUG_SLEEP_MS): a bounded device sleep on the comm stream at every fork, so a
  // stalled collective can be staged on one GPU (it is captured into the step graph like the rest)
  int debug_sleep_ms = 0;
  // one event per watched cycle (WatchState::pending), recycled through a free list
  std::vector<hipEvent_t> watch_evs;
  std::vector<int64_t> watch_free;
  std::atomic<bool> aborted{false};

  hipEvent_t get_event() {
    return events.get([] {
      hipEvent_t e;
      HCB_HIP(hipEventCreate(&e));
      return e;
    });
  }
  // an event recorded behind the work just enqueued on `s`; its token for WatchState::enqueue
  int64_t record_watch(hipStream_t s) {
    int64_t t;
    if (!watch_free.empty()) {
      t = watch_free.back();
      watch_free.pop_back();
    } else {
      hipEvent_t e;
      HCB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      watch_evs.push_back(e);
      t = (int64_t)watch_evs.size() - 1;
    }
    HCB_HIP(hipEventRecord(watch_evs[t], s));
    return t;
  }
  auto watch_done() {
    return [this](int64_t t) { return hipEventQuery(watch_evs[t]) == hipSuccess; };
  }
  auto watch_release() {
    return [this](int64_t t) { watch_free.push_back(t); };
  }
  void flush_timeline(bool block) {
    timeline.flush(
        block, events, [](hipEvent_t e) { return hipEventQuery(e) == hipSuccess; },
        [](hipEvent_t e) { hipEventSynchronize(e); },
        [this](hipEvent_t e) {
          float t = 0.f;
          hipEventElapsedTime(&t, base_ev, e);
          return (double)t;
        });
  }
};

hcb::comm::HandleTable<Comm> g_comms;

Comm* get(int64_t h) {
  Comm* c = g_comms.get(h);
  TORCH_CHECK(c != nullptr, "hcb_comm: invalid communicator handle ", h);
  return c;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) return false;
  return st == hipStreamCaptureStatusActive;
}

// ncclCommAbort can itself wait for work already queued on the comm stream (measured: with a
// stalled step queued it returned only once that step had drained), so it runs on a detached
// thread and the process exits within a bounded time either way; the launcher then stops the
// other ranks (launch/launcher.py fail-fast)
[[noreturn]] void abort_and_exit(Comm* c, int code) {
  c->aborted = true;
  ncclComm_t comm = c->comm;
  c->comm = nullptr;
  if (comm) std::thread([comm] { ncclCommAbort(comm); }).detach();
  std::this_thread::sleep_for(std::chrono::seconds(2));
  std::_Exit(code);
}

void watchdog_loop(Comm* c) {
  using hcb::comm::StallWatch;
  while (!c->stop.load()) {
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv.wait_for(lk, std::chrono::milliseconds(500));
    }
    if (c->stop.load()) break;
    auto now = std::chrono::steady_clock::now();
    {
      std::lock_guard<std::mutex> lk(c->mu);
      c->ws.poll_quiet(now, 1.0, c->watch_done(), c->watch_release());
    }
    double waited = 0;
    const StallWatch::Action act = c->ws.watch.evaluate(now, &waited);
    if (act == StallWatch::kIdle || act == StallWatch::kProgress) continue;
    if (waited > 1.0 && c->comm) {  // stalled: only now ask RCCL whether a peer failed
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
        std::fprintf(stderr, "[hcb watchdog] rank %d: RCCL async error: %s -- aborting communicator\n", c->rank,
                     ncclGetErrorString(ae));
        std::fflush(stderr);
        abort_and_exit(c, 18);
      }
    }
    if (act == StallWatch::kWarn) {
      const int64_t cyc = c->ws.watch.completed() + 1;
      bool graph_cycle;
      {
        std::lock_guard<std::mutex> lk(c->mu);
        graph_cycle = c->ws.is_graph_cycle(cyc);
      }
      std::fprintf(stderr,
                   "[hcb watchdog] rank %d: gradient reduction cycle %lld%s (buckets up to #%lld) has not completed "
                   "after %.0f s; one or more ranks may have stalled (HOROVOD_STALL_CHECK_TIME_SECONDS=%.0f)\n",
                   c->rank, (long long)cyc, graph_cycle ? " (graph-replayed step)" : "",
                   (long long)c->ws.watch.last_seq(), waited, c->ws.watch.warn_s());
      std::fflush(stderr);
    } else if (act == StallWatch::kAbort && c->comm) {
      std::fprintf(stderr, "[hcb watchdog] rank %d: stalled for %.0f s > HCB_STALL_ABORT_SECONDS; aborting\n", c->rank,
                   waited);
      std::fflush(stderr);
      abort_and_exit(c, 19);
    }
  }
}

// RCCL transport of the bucket engine: collectives on the comm stream, forked from / joined
// to the caller's stream with events (capturable: they become graph edges).
struct RcclTransport final : hcb::comm::Transport {
  Comm* c;
  hipStream_t cur = nullptr;
  bool cap = false, tl = false;
  hipEvent_t e0 = nullptr;
  explicit RcclTransport(Comm* c_) : c(c_) {}
  void fork() override {
    cur = c10::hip::getCurrentHIPStream().stream();
    HCB_HIP(hipEventRecord(c->fork_ev, cur));
    HCB_HIP(hipStreamWaitEvent(c->stream, c->fork_ev, 0));
    if (cap && c->debug_sleep_ms > 0) hcb::launch_debug_sleep(c->debug_sleep_ms, c->stream);
  }
  void bucket_begin(const hcb::comm::Bucket&) override {
    if (!tl) return;
    e0 = c->get_event();
    HCB_HIP(hipEventRecord(e0, c->stream));
  }
  void reduce_bucket(float* flat, const hcb::comm::Bucket& b, hcb::comm::Wire w, bool avg) override {
    const ncclRedOp_t op = avg ? ncclAvg : ncclSum;
    if (w != hcb::comm::Wire::F32) {
      const int mode = (int)w;  // 1 bf16, 2 fp16
      uint16_t* cb = reinterpret_cast<uint16_t*>(c->cbuf) + b.off;
      hcb::launch_bucket_pack(flat + b.off, cb, b.len, 1.0f, mode, c->stream);
      HCB_NCCL(ncclAllReduce(cb, cb, b.len, w == hcb::comm::Wire::BF16 ? ncclBfloat16 : ncclFloat16, op, c->comm,
                             c->stream));
      hcb::launch_bucket_unpack(cb, flat + b.off, b.len, 1.0f, mode, c->stream);
    } else {
      HCB_NCCL(ncclAllReduce(flat + b.off, flat + b.off, b.len, ncclFloat32, op, c->comm, c->stream));
    }
  }
  void bucket_end(const hcb::comm::Bucket& b, hcb::comm::Wire w) override {
    if (!tl) return;
    hipEvent_t e1 = c->get_event();
    HCB_HIP(hipEventRecord(e1, c->stream));
    c->timeline.record({w != hcb::comm::Wire::F32 ? "PACK_ALLREDUCE_UNPACK" : "ALLREDUCE", b.seq,
                        b.len * hcb::comm::wire_bytes(w), e0, e1});
  }
  void join() override {
    HCB_HIP(hipEventRecord(c->join_ev, c->stream));
    HCB_HIP(hipStreamWaitEvent(cur, c->join_ev, 0));
    joined = true;
  }
  // the overlap form records the join event without waiting on it: join_() consumes it later
  void mark_cycle_end(int64_t) override {
    if (!joined) HCB_HIP(hipEventRecord(c->join_ev, c->stream));
    joined = false;
  }
  bool joined = false;
};

// ------------------------------------------------------------------------- ops
Tensor unique_id() {
  ncclUniqueId id;
  HCB_NCCL(ncclGetUniqueId(&id));
  Tensor t = at::empty({(int64_t)sizeof(id)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &id, sizeof(id));
  return t;
}

int64_t create(const Tensor& uid, int64_t rank, int64_t world, int64_t device) {
  TORCH_CHECK(uid.numel() == (int64_t)sizeof(ncclUniqueId) && uid.scalar_type() == at::kByte && !uid.is_cuda(),
              "hcb_comm.create: uid must be a CPU uint8 tensor of ", sizeof(ncclUniqueId), " bytes");
  auto c = std::make_unique<Comm>();
  c->rank = (int)rank;
  c->world = (int)world;
  c->device = (int)device;
  HCB_HIP(hipSetDevice(c->device));
  ncclUniqueId id;
  std::memcpy(&id, uid.data_ptr(), sizeof(id));
  HCB_NCCL(ncclCommInitRank(&c->comm, c->world, id, c->rank));
  int prio_lo = 0, prio_hi = 0;
  HCB_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  // communication at high priority so its few kernels are not queued behind compute
  HCB_HIP(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi));
  HCB_HIP(hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
  HCB_HIP(hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming));
  HCB_HIP(hipEventCreate(&c->base_ev));
  HCB_HIP(hipEventRecord(c->base_ev, c->stream));
  if (const char* tl = std::getenv("HOROVOD_TIMELINE")) {
    if (*tl) {
      std::string p(tl);
      if (c->world > 1) p += "." + std::to_string(c->rank);
      c->timeline_path = p;
      c->tl_file.open(p);
      c->timeline.open(&c->tl_file, c->rank);
    }
  }
  c->ws.watch.configure(env_double("HOROVOD_STALL_CHECK_TIME_SECONDS", 60.0), env_double("HCB_STALL_ABORT_SECONDS", 0.0));
  {
    const double fb = env_double("HOROVOD_FUSION_THRESHOLD", 128.0 * 1024 * 1024);
    c->fusion_bytes = fb > 0 ? (int64_t)fb : 0;
  }
  c->debug_sleep_ms = (int)std::min(10000.0, std::max(0.0, env_double("HCB_COMM_DEBUG_SLEEP_MS", 0.0)));
  Comm* raw = c.get();
  if (env_double("HCB_COMM_WATCHDOG", 1.0) != 0.0) raw->wd = std::thread(watchdog_loop, raw);
  return g_comms.add(std::move(c));
}

void destroy(int64_t h) {
  std::unique_ptr<Comm> c = g_comms.take(h);
  if (!c) return;
  c->stop = true;
  c->cv.notify_all();
  if (c->wd.joinable()) c->wd.join();
  hipStreamSynchronize(c->stream);
  c->flush_timeline(true);
  c->timeline.close();
  if (c->tl_file.is_open()) c->tl_file.close();
  if (c->comm) ncclCommDestroy(c->comm);
  c->events.drain([](hipEvent_t e) { hipEventDestroy(e); });
  hipEventDestroy(c->fork_ev);
  hipEventDestroy(c->join_ev);
  hipEventDestroy(c->base_ev);
  for (hipEvent_t e : c->watch_evs) hipEventDestroy(e);
  if (c->cbuf) hipFree(c->cbuf);
  hipStreamDestroy(c->stream);
}

// fork the comm stream off the caller's stream
hipStream_t fork(Comm* c) {
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  HCB_HIP(hipEventRecord(c->fork_ev, cur));
  HCB_HIP(hipStreamWaitEvent(c->stream, c->fork_ev, 0));
  return cur;
}
void join(Comm* c, hipStream_t cur) {
  HCB_HIP(hipEventRecord(c->join_ev, c->stream));
  HCB_HIP(hipStreamWaitEvent(cur, c->join_ev, 0));
}

void allreduce_(int64_t h, const Tensor& t, bool average) {
  Comm* c = get(h);
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "hcb_comm.allreduce_: contiguous GPU tensor");
  TORCH_CHECK(c->comm, "hcb_comm: communicator aborted");
  hipStream_t cur = fork(c);
  HCB_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), average ? ncclAvg : ncclSum,
                         c->comm, c->stream));
  join(c, cur);
}

void broadcast_(int64_t h, const Tensor& t, int64_t root) {
  Comm* c = get(h);
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "hcb_comm.broadcast_: contiguous GPU tensor");
  hipStream_t cur = fork(c);
  HCB_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), (int)root, c->comm, c->stream));
  join(c, cur);
}

void allgather_(int64_t h, const Tensor& in, const Tensor& out) {
  Comm* c = get(h);
  TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "hcb_comm.allgather_");
  TORCH_CHECK(out.numel() == in.numel() * c->world && in.scalar_type() == out.scalar_type(), "hcb_comm.allgather_: sizes");
  hipStream_t cur = fork(c);
  HCB_NCCL(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_type(in), c->comm, c->stream));
  join(c, cur);
}

void reduce_scatter_(int64_t h, const Tensor& in, const Tensor& out, bool average) {
  Comm* c = get(h);
  TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "hcb_comm.reduce_scatter_");
  TORCH_CHECK(in.numel() == out.numel() * c->world && in.scalar_type() == out.scalar_type(), "hcb_comm.reduce_scatter_: sizes");
  hipStream_t cur = fork(c);
  HCB_NCCL(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_type(in), average ? ncclAvg : ncclSum,
                             c->comm, c->stream));
  join(c, cur);
}

// Bucketed allreduce of the flat fp32 gradient buffer.
// ranges: int64 CPU tensor [nr][2] of (offset, length) in elements; each range is cut into
// buckets of at most `fusion_bytes` wire bytes (<= 0: the HOROVOD_FUSION_THRESHOLD default
// read at create()), issued in order on the comm stream.
// compress: 0 none (fp32), 1 bf16, 2 fp16 (IEEE half; Horovod Compression.fp16).
void bucket_impl(int64_t h, const Tensor& flat, const Tensor& buckets, int64_t compress, double scale, bool average,
                 bool do_join, int64_t fusion_bytes) {
  Comm* c = get(h);
  TORCH_CHECK(c->comm, "hcb_comm: communicator aborted");
  TORCH_CHECK(flat.is_cuda() && flat.is_contiguous() && flat.scalar_type() == at::kFloat,
              "hcb_comm.bucket_allreduce_: flat fp32 GPU buffer");
  TORCH_CHECK(!buckets.is_cuda() && buckets.scalar_type() == at::kLong && buckets.dim() == 2 && buckets.size(1) == 2,
              "hcb_comm.bucket_allreduce_: buckets int64 [n][2] on CPU");
  TORCH_CHECK(compress >= 0 && compress <= 2, "hcb_comm.bucket_allreduce_: compress must be 0 (none), 1 (bf16) or 2 (fp16)");
  TORCH_CHECK(scale == 1.0, "hcb_comm.bucket_allreduce_: scale is folded into the optimizer; pass 1.0");
  const at::Tensor bc = buckets.contiguous();  // keep the (possibly copied) table alive while it is read
  const int64_t* bk = bc.data_ptr<int64_t>();
  const int64_t nb = buckets.size(0);
  const int64_t n = flat.numel();
  for (int64_t i = 0; i < nb; ++i)
    TORCH_CHECK(bk[2 * i] >= 0 && bk[2 * i + 1] > 0 && bk[2 * i] + bk[2 * i + 1] <= n, "hcb_comm: bucket out of range");
  std::lock_guard<std::mutex> call_lk(c->mu);  // excludes the watchdog's (rare) event query
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  const bool cap = capturing(cur);
  if (!cap) c->flush_timeline(false);
  if (!cap && c->wd.joinable())
    c->ws.enter(c->watch_done(), c->watch_release());
  else
    c->ws.last_call = std::chrono::steady_clock::now();
  if (const size_t grow = hcb::comm::scratch_bytes(c->cbuf_bytes, n, (hcb::comm::Wire)compress)) {
    TORCH_CHECK(!cap, "hcb_comm: first compressed reduction must run outside graph capture");
    HCB_HIP(hipStreamSynchronize(c->stream));
    if (c->cbuf) HCB_HIP(hipFree(c->cbuf));
    c->cbuf = nullptr;
    c->cbuf_bytes = 0;
    HCB_HIP(hipMalloc(&c->cbuf, grow));
    c->cbuf_bytes = grow;
  }
  if (!c->engine) {
    c->transport = std::make_unique<RcclTransport>(c);
    c->engine = std::make_unique<hcb::comm::BucketEngine>(c->transport.get());
  }
  auto* tr = static_cast<RcclTransport*>(c->transport.get());
  tr->cap = cap;
  tr->tl = c->timeline.is_open() && !cap;
  std::vector<hcb::comm::Bucket> issued =
      c->engine->submit(flat.data_ptr<float>(), n, bk, nb, (hcb::comm::Wire)compress, average,
                 fusion_bytes > 0 ? fusion_bytes : c->fusion_bytes, do_join);
  c->buckets_issued += (int64_t)issued.size();
  if (!cap && c->wd.joinable()) c->ws.enqueue(c->buckets_issued - 1, false, c->record_watch(c->stream));
  c->cycle++;
}

void bucket_allreduce_(int64_t h, const Tensor& flat, const Tensor& buckets, int64_t compress, double scale,
                       bool average) {
  bucket_impl(h, flat, buckets, compress, scale, average, true, 0);
}

// Overlap form: the comm stream waits for the caller's stream (everything enqueued so far,
// e.g. a replayed backward segment) but the caller does NOT wait for the reduction; call
// join_() before consuming the reduced buffer. Successive async calls queue in order on the
// comm stream, so one join covers them all.
void bucket_allreduce_async_(int64_t h, const Tensor& flat, const Tensor& buckets, int64_t compress, double scale,
                             bool average) {
  bucket_impl(h, flat, buckets, compress, scale, average, false, 0);
}

// Per-step heartbeat of the graph-replayed data-parallel step (call right after the replay, on
// the stream it was launched on, never inside a capture). The collectives of a captured step
// make no host call when replayed, so without this the watchdog would never learn about them:
// record a watch event of this step's own behind it (the graph's comm branch joins the capture
// stream before the graph ends, so the event completes only once every reduction of the step
// has) and enqueue one watch cycle. As for eager reductions, completion is observed without
// blocking on the CALLER's thread (every earlier mark whose event has finished, oldest first) or,
// once the caller has been quiet for > 1 s (blocked on a hung step), by the watchdog thread.
void step_mark(int64_t h) {
  Comm* c = get(h);
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  TORCH_CHECK(!capturing(cur), "hcb_comm.step_mark: call after a replay, not inside a capture");
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->wd.joinable()) {
    c->ws.last_call = std::chrono::steady_clock::now();
    c->ws.marks++;
    return;
  }
  c->ws.enter(c->watch_done(), c->watch_release());
  c->ws.enqueue(c->buckets_issued - 1, true, c->record_watch(cur));
}
int64_t steps_marked(int64_t h) {
  Comm* c = get(h);
  std::lock_guard<std::mutex> lk(c->mu);
  return c->ws.marks;
}

int64_t buckets_issued(int64_t h) { return get(h)->buckets_issued; }
int64_t fusion_threshold(int64_t h) { return get(h)->fusion_bytes; }
void set_fusion_threshold(int64_t h, int64_t bytes) { get(h)->fusion_bytes = bytes; }

void join_(int64_t h) {
  Comm* c = get(h);
  HCB_HIP(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), c->join_ev, 0));
}

void barrier(int64_t h) {
  Comm* c = get(h);
  Tensor t = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, c->device));
  allreduce_(h, t, false);
  HCB_HIP(hipStreamSynchronize(c10::hip::getCurrentHIPStream().stream()));
}

// ------------------------------------------------------------ one-shot xGMI allreduce
// IPC-shared staging regions (csrc/kernels/xgmi.hip has the protocol). Independent of the
// RCCL communicator: handles are exchanged by the Python side over torch.distributed.
struct Xgmi {
  hcb::comm::XgmiBook book;         // rank / world / capacity / peer mapping (comm/host.h)
  int device = 0;
  unsigned spin = 1u << 25;         // bounded-wait iterations
  float* region = nullptr;          // own region: 2 slots + flags
  unsigned* err = nullptr;          // device error word (spin timeout)
};
hcb::comm::HandleTable<Xgmi> g_xgmi;

Xgmi* xget(int64_t h) {
  Xgmi* x = g_xgmi.get(h);
  TORCH_CHECK(x != nullptr, "hcb_comm: invalid xgmi handle ", h);
  return x;
}

int64_t xgmi_create(int64_t rank, int64_t world, int64_t cap, int64_t device) {
  const std::string bad = hcb::comm::XgmiBook::check_create(rank, world, cap, hcb::xgmi_max_ranks());
  TORCH_CHECK(bad.empty(), "hcb_comm.xgmi_create: ", bad);
  auto x = std::make_unique<Xgmi>();
  x->device = (int)device;
  HCB_HIP(hipSetDevice(x->device));
  const size_t bytes = hcb::comm::XgmiBook::region_bytes(cap);
  // uncached (fine-grained) device memory: peers on OTHER GPUs spin on the ready / epoch words
  // and read the slots over xGMI while this GPU is still running; coarse-grained memory is only
  // coherent across devices at kernel boundaries
  HCB_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&x->region), bytes, hipDeviceMallocUncached));
  x->spin = 1u << 25;  // bounded waits: ~7 s of s_sleep(8) before a dead peer is reported
  HCB_HIP(hipMemset(x->region, 0, bytes));
  HCB_HIP(hipMalloc(&x->err, 4));
  HCB_HIP(hipMemset(x->err, 0, 4));
  HCB_HIP(hipDeviceSynchronize());
  x->book.init((int)rank, (int)world, cap, x->region);
  return g_xgmi.add(std::move(x));
}

Tensor xgmi_handle(int64_t h) {
  Xgmi* x = xget(h);
  hipIpcMemHandle_t mh;
  HCB_HIP(hipIpcGetMemHandle(&mh, x->region));
  Tensor t = at::empty({(int64_t)sizeof(mh)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &mh, sizeof(mh));
  return t;
}

void xgmi_open(int64_t h, const Tensor& handles) {
  Xgmi* x = xget(h);
  TORCH_CHECK(!handles.is_cuda() && handles.scalar_type() == at::kByte && handles.dim() == 2 &&
                  handles.size(0) == x->book.world && handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
              "hcb_comm.xgmi_open: handles uint8 [world][", sizeof(hipIpcMemHandle_t), "] on CPU");
  const at::Tensor hc = handles.contiguous();
  HCB_HIP(hipSetDevice(x->device));
  for (int r = 0; r < x->book.world; ++r) {
    if (r == x->book.rank) continue;
    hipIpcMemHandle_t mh;
    std::memcpy(&mh, hc.data_ptr<uint8_t>() + (size_t)r * sizeof(mh), sizeof(mh));
    void* p = nullptr;
    HCB_HIP(hipIpcOpenMemHandle(&p, mh, hipIpcMemLazyEnablePeerAccess));
    x->book.set_peer(r, p);
  }
}

void xgmi_allreduce_(int64_t h, const Tensor& t, double scale) {
  Xgmi* x = xget(h);
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat,
              "hcb_comm.xgmi_allreduce_: contiguous fp32 GPU tensor");
  const std::string bad = x->book.check_reduce(t.numel());
  TORCH_CHECK(bad.empty(), "hcb_comm.xgmi_allreduce_: ", bad);
  if (t.numel() == 0) return;
  std::vector<const float*> b;
  for (void* p : x->book.peers) b.push_back(static_cast<const float*>(p));
  hcb::launch_xgmi_allreduce(b.data(), x->book.world, x->book.rank, t.data_ptr<float>(), t.data_ptr<float>(),
                             t.numel(), x->book.cap, (float)scale, x->err, x->spin,
                             c10::hip::getCurrentHIPStream().stream());
}

int64_t xgmi_error(int64_t h) {
  Xgmi* x = xget(h);
  unsigned v = 0;
  HCB_HIP(hipMemcpy(&v, x->err, 4, hipMemcpyDeviceToHost));
  return (int64_t)v;
}

void xgmi_destroy(int64_t h) {
  std::unique_ptr<Xgmi> x = g_xgmi.take(h);
  if (!x) return;
  hipSetDevice(x->device);
  hipDeviceSynchronize();
  for (int r = 0; r < x->book.world; ++r)
    if (x->book.opened[r]) hipIpcCloseMemHandle(x->book.peers[r]);
  hipFree(x->region);
  hipFree(x->err);
}

int64_t comm_rank(int64_t h) { return get(h)->rank; }
// rank count as the RCCL communicator reports it (not the value it was created with), so a
// benchmark can prove how many ranks its reductions really spanned
int64_t comm_size(int64_t h) {
  Comm* c = get(h);
  TORCH_CHECK(c->comm, "hcb_comm: communicator aborted");
  int n = 0;
  HCB_NCCL(ncclCommCount(c->comm, &n));
  return n;
}

void abort_comm(int64_t h) {
  Comm* c = get(h);
  if (c->comm) {
    ncclCommAbort(c->comm);
    c->comm = nullptr;
  }
}

std::string version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v);
}

}  // namespace

TORCH_LIBRARY(hcb_comm, m) {
  m.def("unique_id() -> Tensor", unique_id);
  m.def("create(Tensor uid, int rank, int world, int device) -> int", create);
  m.def("destroy(int h) -> ()", destroy);
  m.def("allreduce_(int h, Tensor(a!) t, bool average) -> ()", allreduce_);
  m.def("broadcast_(int h, Tensor(a!) t, int root) -> ()", broadcast_);
  m.def("allgather_(int h, Tensor input, Tensor(a!) output) -> ()", allgather_);
  m.def("reduce_scatter_(int h, Tensor input, Tensor(a!) output, bool average) -> ()", reduce_scatter_);
  m.def("bucket_allreduce_(int h, Tensor(a!) flat, Tensor buckets, int compress, float scale, bool average) -> ()",
        bucket_allreduce_);
  m.def("bucket_allreduce_async_(int h, Tensor(a!) flat, Tensor buckets, int compress, float scale, bool average) -> ()",
        bucket_allreduce_async_);
  m.def("join_(int h) -> ()", join_);
  m.def("buckets_issued(int h) -> int", buckets_issued);
  m.def("step_mark(int h) -> ()", step_mark);
  m.def("steps_marked(int h) -> int", steps_marked);
  m.def("fusion_threshold(int h) -> int", fusion_threshold);
  m.def("set_fusion_threshold(int h, int bytes) -> ()", set_fusion_threshold);
  m.def("barrier(int h) -> ()", barrier);
  m.def("rank(int h) -> int", comm_rank);
  m.def("size(int h) -> int", comm_size);
  m.def("abort(int h) -> ()", abort_comm);
  m.def("version() -> str", version);
  m.def("xgmi_create(int rank, int world, int cap, int device) -> int", xgmi_create);
  m.def("xgmi_handle(int h) -> Tensor", xgmi_handle);
  m.def("xgmi_open(int h, Tensor handles) -> ()", xgmi_open);
  m.def("xgmi_allreduce_(int h, Tensor(a!) t, float scale) -> ()", xgmi_allreduce_);
  m.def("xgmi_error(int h) -> int", xgmi_error);
  m.def("xgmi_destroy(int h) -> ()", xgmi_destroy);
}
