// One-shot peer-to-peer allreduce over xGMI for small buffers (SURVEY.md §2.3 "optional
// hand-written one-/two-shot xGMI allreduce via IPC peer pointers"; the reference's small
// Horovod/MPI_Allreduce messages, run-tf-sing-ucx-openmpi.sh:105).
//
// Every rank owns an IPC-exported staging region   [slot 0 | slot 1 | flags]:
//   slot e%2  (cap floats)  this rank's contribution of epoch e
//   flags     ready (u32, the last epoch whose slot is complete), epoch (u32, local),
//             arrive counter (u32, local)
// and maps every peer's region (hipIpcOpenMemHandle). One call = two kernels on the caller's
// stream, epoch kept on the device (graph-replay safe):
//   push:   wait until every peer published epoch e-1 (so it has finished READING my slot of
//           epoch e-2, the one about to be overwritten), copy my input into slot e%2,
//           system-scope release, the last workgroup to arrive publishes ready = e;
//   reduce: wait until every peer published epoch e, then out = scale * sum over ranks of
//           their slot e%2, read with system-scope (cache-bypassing) loads; the last
//           workgroup advances the device epoch.
// Ranks never write into a peer's memory; a peer's data is only read after its release.
// Spins are bounded (Xgmi::spin iterations of s_sleep(8), ~0.2 us each at 2.4 GHz; default
// 2^25 ~ 7 s): on timeout the kernel raises the error word, POISONS its output with NaN (so a
// reduction that did not synchronise can never pass for a good one: the loss goes NaN) and
// completes, so a dead peer can never leave a wave running on the GPU. The host side checks
// the error word (NativeReducer.check_errors) and raises.
#include "common.h"
#include "kernels.h"

namespace hcb {

constexpr int XGMI_MAX_RANKS = 8;

struct XgmiPtrs {
  const float* base[XGMI_MAX_RANKS];  // every rank's region (own included)
};

__device__ __forceinline__ unsigned xg_load_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread 0 waits until every rank's ready word reaches `want`; returns false on timeout
__device__ bool xg_wait_all(const XgmiPtrs& P, int R, size_t flag_off, unsigned want, unsigned* err,
                            unsigned spin) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    for (int r = 0; r < R; ++r) {
      const unsigned* f = reinterpret_cast<const unsigned*>(P.base[r] + flag_off);
      unsigned it = 0;
      while ((int)(xg_load_flag(f) - want) < 0) {
        __builtin_amdgcn_s_sleep(8);
        if (++it > spin) {
          atomicOr(err, 1u);
          ok = 0;
          break;
        }
      }
      if (!ok) break;
    }
  }
  __syncthreads();
  return ok != 0;
}

__global__ __launch_bounds__(256) void xgmi_push_kernel(XgmiPtrs P, int R, int rank, const float* __restrict__ in,
                                                        int64_t n, int64_t cap, unsigned* err, unsigned spin) {
  const size_t flag_off = (size_t)2 * cap;  // in floats
  float* mine = const_cast<float*>(P.base[rank]);
  unsigned* myflags = reinterpret_cast<unsigned*>(mine + flag_off);  // [0] ready [1] epoch [2] arrive
  const unsigned e = __hip_atomic_load(myflags + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  if (e > 1) xg_wait_all(P, R, flag_off, e - 1, err, spin);
  float* slot = mine + (size_t)(e & 1) * cap;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<float4*>(slot)[i] = reinterpret_cast<const float4*>(in)[i];
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    slot[i] = in[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(myflags + 2, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {  // last workgroup: every copy is complete and released
      __hip_atomic_store(myflags + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(myflags + 0, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(256) void xgmi_reduce_kernel(XgmiPtrs P, int R, int rank, float* __restrict__ out,
                                                          int64_t n, int64_t cap, float scale, unsigned* err,
                                                          unsigned spin) {
  const size_t flag_off = (size_t)2 * cap;
  float* mine = const_cast<float*>(P.base[rank]);
  unsigned* myflags = reinterpret_cast<unsigned*>(mine + flag_off);
  const unsigned e = __hip_atomic_load(myflags + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const bool synced = xg_wait_all(P, R, flag_off, e, err, spin) &&
                      __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
  const size_t so = (size_t)(e & 1) * cap;
  if (!synced) scale = __builtin_nanf("");  // poison: never return an unsynchronised sum
  const int64_t n2 = n / 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int r = 0; r < XGMI_MAX_RANKS; ++r) {
      if (r >= R) break;
      // system-scope 8-byte loads: the peer's slot is re-read every other epoch, so it must
      // not be served from a cache line filled two epochs ago
      const unsigned long long* src = reinterpret_cast<const unsigned long long*>(P.base[r] + so) + i;
      const unsigned long long v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      a0 += __uint_as_float((unsigned)(v & 0xffffffffu));
      a1 += __uint_as_float((unsigned)(v >> 32));
    }
    out[2 * i] = a0 * scale;
    out[2 * i + 1] = a1 * scale;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    float a = 0.f;
    for (int r = 0; r < R; ++r)
      a += __hip_atomic_load(P.base[r] + so + (n - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    out[n - 1] = a * scale;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(myflags + 2, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {  // last workgroup: this rank is done with epoch e
      __hip_atomic_store(myflags + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(myflags + 1, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int xgmi_max_ranks() { return XGMI_MAX_RANKS; }

void launch_xgmi_allreduce(const float* const* bases, int R, int rank, const float* in, float* out, int64_t n,
                           int64_t cap, float scale, unsigned* err, unsigned spin, hipStream_t st) {
  XgmiPtrs P{};
  for (int r = 0; r < R && r < XGMI_MAX_RANKS; ++r) P.base[r] = bases[r];
  // few workgroups: the push / reduce are bandwidth-light and every workgroup's thread 0 spins
  int64_t want = (n + 256 * 8 - 1) / (256 * 8);
  const int grid = (int)(want < 1 ? 1 : (want > 64 ? 64 : want));
  hipLaunchKernelGGL(xgmi_push_kernel, dim3(grid), dim3(256), 0, st, P, R, rank, in, n, cap, err, spin);
  hipLaunchKernelGGL(xgmi_reduce_kernel, dim3(grid), dim3(256), 0, st, P, R, rank, out, n, cap, scale, err, spin);
}

}  // namespace hcb
