// Minimal fork/join HIP-graph ordering checks, shaped like the training step's graph.
//
//   hipcc --offload-arch=gfx950 -O2 tools/graph_fork_repro.hip -o tools/graph_fork_repro
//   DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 tools/graph_fork_repro <replays> <mode>
//
// mode 0 "fork": k_seed bumps a device epoch e and fills x = e; a forked branch computes
//   y = x + 1 through a dependent chain, the main branch computes z = 2x meanwhile; after the
//   join k_check counts elements with y != e + 1 or z != 2e.
// mode 1 "segments": the data-parallel step's pattern -- a long chain of dependent kernels on
//   the main stream (a = a + 1, 256 launches) with, every 32 launches, a fork of the comm stream
//   off the main stream (ONE fork event and ONE join event, re-recorded per segment, as in
//   csrc/comm/comm.cpp), a kernel on the comm stream over a separate buffer, the join event
//   recorded without a wait; the main stream waits on the last join at the end.
// mode 2: mode 1 with an EMPTY comm branch (the HCB_COMM_SKIP_RCCL=1 shape).
// mode 3 / 4: modes 1 / 2 with a highest-priority comm stream (as the engine creates it).
// mode 5: mode 2 plus, in every link of the chain, a hipMemsetAsync node zeroing an accumulator
//   that the next kernel adds into (the training step's zero-initialised BN accumulators /
//   split-K dx buffers: torch.zeros inside the capture); mode 6: the same without the forks.
// mode 7: the dependent chain with a CROSS-XCD dependency: link k+1 reads element i + 256 of
//   link k's output, written by the NEXT workgroup (blockIdx + 1: the neighbouring XCD of the
//   8), so a stale per-XCD L2 line (a missing write-back / invalidate between two graph kernels)
//   shows up; no forks. mode 8: mode 7 with a memset node + accumulate per link.
// mode 9: a chain through a SCALAR value: link k reads s_k with a wave-uniform load (an s_load
//   through the scalar cache) that link k-1 wrote, fills x with it and writes s_{k+1} = s_k + 1;
//   a scalar cache left uninvalidated between two graph kernels reads a stale s_k.
// mode 10 / 11: the training step's bias-gradient pattern (launch_colsum2, csrc/kernels/misc.hip):
//   a kernel dirties a float region, hipMemsetAsync(region, 0, bytes) zeroes it, a consumer
//   counts the elements that are not zero -- mode 10 with 1001 floats (4004 bytes, not a multiple
//   of 8 / 16: the fc bias of a 1001-class head), mode 11 with 1024 floats (4096 bytes). The
//   region sits 256-byte aligned inside a larger allocation, as the bias slice of the flat
//   gradient buffer does. mode 12: mode 10 with EAGER work between the replays (a kernel and a
//   hipMemsetAsync with another destination, size and value on the same stream -- what a training
//   loop does between two step graphs: loss copies, statistics); mode 13: eager kernels only;
//   mode 14: eager memsets only. mode 15: the step graph's SIZE around the memset: 320 kernel
//   nodes with 512-byte kernel arguments (the conv kernels pass a ~0.5 KB ConvParams by value)
//   before and after one dirty / memset / check link, per replay.
// Any ordering violation (a kernel started before its predecessor finished) or cross-XCD
// visibility gap shows up as a nonzero error count.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      std::exit(2);                                                                               \
    }                                                                                             \
  } while (0)

__global__ void k_seed(const unsigned* epoch, float* x, int n) {
  const float e = (float)((*epoch + 1) & 0xffff);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = e;
}
__global__ void k_bump(unsigned* epoch) { *epoch += 1; }
__global__ void k_copy_add(const float* a, float* b, int n, float add) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = a[i] + add;
}
__global__ void k_scale(const float* a, float* b, int n, float s) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = a[i] * s;
}
__global__ void k_rot_add(const float* a, float* b, int n, int shift) {  // b[i] = a[i + shift] + 1
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = a[(i + shift) % n] + 1.f;
}
__global__ void k_rot_accum(const float* a, float* acc, int n, int shift) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    acc[i] += a[(i + shift) % n] + 1.f;
}
__global__ void k_scalar_link(const float* s_in, float* s_out, float* x, int n) {
  const float v = s_in[0];  // uniform address: scalar load
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = v;
  if (blockIdx.x == 0 && threadIdx.x == 0) s_out[0] = v + 1.f;
}
__global__ void k_accum(const float* a, float* acc, int n) {  // acc = 0 (memset) + a + 1
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) acc[i] += a[i] + 1.f;
}
__global__ void k_dirty(float* r, int n, const unsigned* epoch) {  // any non-zero pattern
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    r[i] = 1.0e30f + (float)(*epoch & 0xff) + (float)i;
}
struct BigArgs {
  float* dst;
  int n;
  int pad[125];  // 512 bytes of kernel arguments
};
__global__ void k_big(BigArgs a) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x)
    a.dst[i] += (float)a.pad[i & 63];
}
__global__ void k_count_nonzero(const float* r, int n, unsigned* errors) {
  unsigned bad = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) bad += r[i] != 0.f;
  if (bad) atomicAdd(errors, bad);
}
__global__ void k_check(const unsigned* epoch, const float* y, float yadd, const float* z, float zmul, int n,
                        unsigned* errors) {
  const float e = (float)(*epoch & 0xffff);
  unsigned bad = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    bad += (y[i] != e + yadd) + (z != nullptr && z[i] != zmul * e);
  if (bad) atomicAdd(errors, bad);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 1000;
  const int mode = argc > 2 ? std::atoi(argv[2]) : 0;
  const int n = mode == 0 ? 1 << 22 : 1 << 18;
  float *x, *t0, *t1, *y, *z;
  unsigned *epoch, *errors;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&t0, n * 4));
  CK(hipMalloc(&t1, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&z, n * 4));
  CK(hipMalloc(&epoch, 4));
  CK(hipMalloc(&errors, 4));
  CK(hipMemset(epoch, 0, 4));
  CK(hipMemset(errors, 0, 4));
  CK(hipMemset(z, 0, n * 4));
  hipStream_t s, c;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (mode >= 3) {  // the engine's comm stream: highest priority
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&c, hipStreamNonBlocking, hi));
  } else {
    CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  }
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));

  const dim3 g(mode == 0 ? 1024 : 256), b(256);
  const int chain = 256, seg = 32;
  hipGraph_t graph;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(k_seed, g, b, 0, s, epoch, x, n);
  hipLaunchKernelGGL(k_bump, dim3(1), dim3(1), 0, s, epoch);
  if (mode == 15) {
    const int nf = 1001;
    float* region = z + 4096;
    BigArgs ba{};
    ba.dst = t1;
    ba.n = 4096;
    for (int k = 0; k < 125; ++k) ba.pad[k] = k;
    for (int k = 0; k < 320; ++k) hipLaunchKernelGGL(k_big, dim3(16), dim3(256), 0, s, ba);
    hipLaunchKernelGGL(k_dirty, dim3(4), dim3(256), 0, s, region, nf, epoch);
    CK(hipMemsetAsync(region, 0, (size_t)nf * 4, s));
    hipLaunchKernelGGL(k_count_nonzero, dim3(4), dim3(256), 0, s, region, nf, errors);
    for (int k = 0; k < 320; ++k) hipLaunchKernelGGL(k_big, dim3(16), dim3(256), 0, s, ba);
  } else if (mode >= 10 && mode <= 14) {
    const int nf = mode == 11 ? 1024 : 1001;
    float* region = z + 4096;  // 16 KiB into the allocation: 256-byte aligned
    for (int k = 0; k < 64; ++k) {  // 64 dirty / zero / check links per replay
      hipLaunchKernelGGL(k_dirty, dim3(4), dim3(256), 0, s, region, nf, epoch);
      CK(hipMemsetAsync(region, 0, (size_t)nf * 4, s));
      hipLaunchKernelGGL(k_count_nonzero, dim3(4), dim3(256), 0, s, region, nf, errors);
    }
  } else if (mode == 0) {
    CK(hipEventRecord(fork, s));
    CK(hipStreamWaitEvent(c, fork, 0));
    hipLaunchKernelGGL(k_copy_add, g, b, 0, c, x, t0, n, 0.25f);
    hipLaunchKernelGGL(k_copy_add, g, b, 0, c, t0, t1, n, 0.25f);
    hipLaunchKernelGGL(k_copy_add, g, b, 0, c, t1, y, n, 0.5f);
    CK(hipEventRecord(join, c));
    hipLaunchKernelGGL(k_scale, g, b, 0, s, x, z, n, 2.f);
    CK(hipStreamWaitEvent(s, join, 0));
    hipLaunchKernelGGL(k_check, g, b, 0, s, epoch, y, 1.f, z, 2.f, n, errors);
  } else {
    float* a = x;
    float* o = t0;
    const bool memset_mode = mode == 5 || mode == 6 || mode == 8;
    const bool rot = mode == 7 || mode == 8;
    const bool scal = mode == 9;
    if (scal) hipLaunchKernelGGL(k_copy_add, dim3(1), dim3(64), 0, s, x, t1, 64, 0.f);  // s_0 = e (t1[0])
    for (int k = 0; k < chain; ++k) {
      if (scal) {
        // s_k lives in t1[k & 1]... alternate two scalar slots: read slot k&1, write the other
        hipLaunchKernelGGL(k_scalar_link, g, b, 0, s, t1 + (k & 1), t1 + ((k + 1) & 1), o, n);
      } else if (memset_mode) {  // o = 0 by a memset node, then o += a + 1
        CK(hipMemsetAsync(o, 0, n * 4, s));
        if (rot)
          hipLaunchKernelGGL(k_rot_accum, g, b, 0, s, a, o, n, 256);
        else
          hipLaunchKernelGGL(k_accum, g, b, 0, s, a, o, n);
      } else if (rot) {
        hipLaunchKernelGGL(k_rot_add, g, b, 0, s, a, o, n, 256);
      } else {
        hipLaunchKernelGGL(k_copy_add, g, b, 0, s, a, o, n, 1.f);
      }
      float* t = a;
      a = o;
      o = t;
      if ((k + 1) % seg == 0 && mode != 6 && !rot && !scal) {
        CK(hipEventRecord(fork, s));
        CK(hipStreamWaitEvent(c, fork, 0));
        // comm branch: reads the segment's result into a side buffer (like a bucket pack)
        if (mode == 1 || mode == 3) hipLaunchKernelGGL(k_scale, g, b, 0, c, a, z, n, 1.f);
        CK(hipEventRecord(join, c));
      }
    }
    if (!rot && !scal && mode != 6) CK(hipStreamWaitEvent(s, join, 0));
    if (scal)  // the last link filled its buffer with s_255 = e + 255, and wrote s_256 = e + 256
      hipLaunchKernelGGL(k_check, g, b, 0, s, epoch, a, (float)(chain - 1), nullptr, 0.f, n, errors);
    else
      hipLaunchKernelGGL(k_check, g, b, 0, s, epoch, a, (float)chain, nullptr, 0.f, n, errors);
    // z holds the LAST segment's value (e + chain) when the comm branch ran in order
    if (mode == 1 || mode == 3) hipLaunchKernelGGL(k_check, g, b, 0, s, epoch, z, (float)chain, nullptr, 0.f, n, errors);
  }
  CK(hipStreamEndCapture(s, &graph));
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));

  const bool eager_k = mode == 12 || mode == 13, eager_m = mode == 12 || mode == 14;
  for (int it = 0; it < iters; ++it) {
    CK(hipGraphLaunch(exec, s));
    if (eager_k) hipLaunchKernelGGL(k_dirty, dim3(8), dim3(256), 0, s, t1, 2048 + (it & 7), epoch);
    if (eager_m) CK(hipMemsetAsync(t0 + 64 * (it & 15), 0x5a, (size_t)(3000 + 4 * (it & 31)), s));
  }
  CK(hipStreamSynchronize(s));
  unsigned host_err = 0, host_epoch = 0;
  CK(hipMemcpy(&host_err, errors, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&host_epoch, epoch, 4, hipMemcpyDeviceToHost));
  const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
  std::printf("graph_fork_repro: mode=%d DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s replays=%d epoch=%u errors=%u\n", mode,
              pc ? pc : "(unset)", iters, host_epoch, host_err);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return host_err == 0 && host_epoch == (unsigned)iters ? 0 : 1;
}
