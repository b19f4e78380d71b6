// Shared main-loop pieces of the implicit-GEMM conv kernels (conv_igemm.hip, conv_p3.hip):
// the division-free implicit-im2col loader, the counted LDS-DMA wait and the bf16x6 MFMA step of
// the fp32 path.
#pragma once
#include "common.h"
#include "kernels.h"

namespace hcb {

// ---- per-thread implicit-im2col address generation, shared by both main loops.
// k-steps are issued strictly in order (kt = 0, 1, 2, ...), so the loader keeps the current
// filter tap / channel offset as wave-uniform state and advances it without divisions. In
// the CBIG path (C % 64 == 0: a 64-deep k-step never straddles a tap) the per-row work is
// two adds, two unsigned compares and a select; invalid rows carry h0 = INT_MIN/2 so the
// bounds test rejects them without a separate flag.
// RP: rows per load pass (threads / (KW / 8)); ESZ: bytes per element (4: fp32 x); KW: channels per
// k-step (64, or 32 for the half-depth stages of the plane GEMMs, conv_p3.hip)
template <int AV, bool CBIG, bool LHSDIL, int RP = 32, int ESZ = 2, int KW = 64>
struct ALoader {
  static constexpr int LPR = KW / 8;  // lanes per tile row
  int h0[AV], w0[AV];
  int rowoff[AV];  // byte offset of (pixel of tap (0,0)) * ldx + lane chunk, may be negative
  int pix[AV];     // generic path: first pixel of the image, -1 = row beyond M
  int tr, ts, tc;  // CBIG: current tap (r, s) and channel offset

  __device__ __forceinline__ void init(const ConvParams& p, int m0, int tid, int chunk) {
    const int PQ = p.P * p.Q;
    tr = 0;
    ts = 0;
    tc = 0;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      int m = m0 + tid / LPR + RP * v;
      if (m < p.M) {
        int n = m / PQ, r = m - n * PQ;
        int pp = r / p.Q, qq = r - pp * p.Q;
        pix[v] = n * p.H * p.W;
        h0[v] = pp * p.stride_h - p.pad_h;
        w0[v] = qq * p.stride_w - p.pad_w;
        rowoff[v] = ((pix[v] + h0[v] * p.W + w0[v]) * p.ldx + chunk * 8) * ESZ;
      } else {
        pix[v] = -1;
        h0[v] = -0x40000000;
        w0[v] = 0;
        rowoff[v] = 0;
      }
    }
  }
  // position the incremental tap state at k-step kt0 (a split-K block's first k-step)
  __device__ __forceinline__ void seek(const ConvParams& p, int kt0) {
    const int k0 = kt0 * KW;
    const int tap = k0 / p.C;
    tc = k0 - tap * p.C;
    tr = tap / p.S;
    ts = tap - tr * p.S;
  }
  // byte offsets of this thread's 16-byte vectors (row v, k-chunk `chunk`) of k-step kt
  __device__ __forceinline__ void offsets(const ConvParams& p, int kt, int chunk, uint32_t (&off)[AV]) {
    if constexpr (CBIG && !LHSDIL) {
      const int dh = tr * p.dil_h, dw = ts * p.dil_w;
      const int uoff = ((dh * p.W + dw) * p.ldx + tc) * ESZ;
      const bool tap_ok = tr < p.R;
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int h = h0[v] + dh, w = w0[v] + dw;
        const bool ok = tap_ok && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
        off[v] = ok ? (uint32_t)(rowoff[v] + uoff) : HCB_OOB;
      }
      // advance to the next KW-channel slab
      tc += KW;
      if (tc >= p.C) {
        tc = 0;
        if (++ts == p.S) {
          ts = 0;
          ++tr;
        }
      }
    } else {
      const int k0 = kt * KW;
      int tap, c, r, s;
      if constexpr (CBIG) {
        tap = k0 / p.C;
        c = k0 - tap * p.C + chunk * 8;
      } else {
        // per-lane k (the chunk): shifts when C is a power of two (the space-to-depth stem's 16
        // channels) instead of a VALU integer division per thread and k-step
        const int k = k0 + chunk * 8;
        if ((p.C & (p.C - 1)) == 0) {
          const int lc = __builtin_ctz((unsigned)p.C);
          tap = k >> lc;
          c = k & (p.C - 1);
        } else {
          tap = k / p.C;
          c = k - tap * p.C;
        }
      }
      if ((p.S & (p.S - 1)) == 0) {
        const int ls = __builtin_ctz((unsigned)p.S);
        r = tap >> ls;
        s = tap & (p.S - 1);
      } else {
        r = tap / p.S;
        s = tap - r * p.S;
      }
      const bool tap_ok = tap < p.R * p.S;
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        int h = h0[v] + r * p.dil_h;
        int w = w0[v] + s * p.dil_w;
        bool ok = tap_ok && pix[v] >= 0 && h >= 0 && w >= 0;
        if constexpr (LHSDIL) {
          ok = ok && (h % p.idil_h == 0) && (w % p.idil_w == 0);
          h /= p.idil_h;
          w /= p.idil_w;
        }
        ok = ok && h < p.H && w < p.W;
        off[v] = ok ? (uint32_t)((pix[v] + h * p.W + w) * p.ldx + c) * (uint32_t)ESZ : HCB_OOB;
      }
    }
  }
};

// HCB_ILV (default on): a ring slot's LDS-DMA refill issues (and, in the register-double-buffered
// plane GEMMs, the next slot's fragment reads) are spread among its MFMAs (sched_group_barrier)
// instead of issued as a burst between the barrier and the first MFMA. An LDS-DMA piece costs ~60 cycles of its wave's issue (MI355X guide, cycle
// constants): six of them after each barrier left every wave of the workgroup -- both waves of a
// SIMD at once, in lockstep behind the barrier -- not issuing MFMAs for ~400 cycles per slot.
#ifndef HCB_ILV
#define HCB_ILV 1
#endif
// sched_group_barrier masks (LLVM AMDGPU IGroupLP)
constexpr int SG_MFMA = 0x008, SG_VMEM = 0x010, SG_DSR = 0x100;
// ND VMEM issues evenly over the first MFMAs, then NR DS reads evenly over the MFMAs up to 5/6 of
// the NM (the compiler orders every fragment read after every LDS-DMA of the block: it cannot prove
// that the slot being refilled is not the one being read, so reads never go before the last piece).
// Without reads the pieces spread over the first half.
template <int NM, int ND, int NR, int I = 0>
__device__ __forceinline__ void ilv_schedule() {
  if constexpr (I < NM) {
    constexpr int DM = NR > 0 ? (NM / 3 > 0 ? NM / 3 : 1) : (NM / 2 > 0 ? NM / 2 : 1);
    constexpr int RE = NM * 5 / 6 > DM ? NM * 5 / 6 : NM, RN = RE - DM > 0 ? RE - DM : 1;
    constexpr int d = I < DM ? (I + 1) * ND / DM - I * ND / DM : 0;
    constexpr int J = I - DM;
    constexpr int r = (J >= 0 && J < RN) ? (J + 1) * NR / RN - J * NR / RN : 0;
    __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
    if constexpr (d > 0) __builtin_amdgcn_sched_group_barrier(SG_VMEM, d, 0);
    if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(SG_DSR, r, 0);
    ilv_schedule<NM, ND, NR, I + 1>();
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace hcb
