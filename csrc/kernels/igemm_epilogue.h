// Shared epilogue of the implicit-GEMM conv kernels: fp32 accumulators -> (fused BN
// statistics from registers) -> LDS staging (padded fp32 rows) -> coalesced 16-byte stores
// with optional beta-accumulate, bias, fp32 output, strided-output pixel remap, and the
// fused BN-backward gating / reduction of a data-grad GEMM (ConvParams::bnb_*).
//
// The fused BN-backward variant (BNB, its own kernel instantiation so the plain kernels keep
// their register budget) fetches z / y / the beta source of a chunk of up to 4 output
// segments at once, the first chunk before the barrier, so the load latency is paid once per
// chunk and overlaps the barrier instead of once per segment.
#pragma once
#include "common.h"
#include "kernels.h"

namespace hcb {

// fused BN-backward epilogue: output segments prefetched per chunk and thread
constexpr int BNB_PREFETCH_CH = 4;

// Bytes of LDS the epilogue needs for a BM x BN tile computed by WM x WN waves. s16: the plain
// bf16-output epilogue without beta / bias stages the tile as 16-bit values (rounded once, the
// same values the fp32 staging would store), half the LDS -- more workgroups per CU on the
// memory-bound short-K layers whose occupancy the staging buffer sets.
constexpr size_t igemm_epilogue_lds(int BM, int BN, int WM, bool s16 = false) {
  return (s16 ? (size_t)BM * (BN + 8) * 2 : (size_t)BM * (BN + 4) * 4) + (size_t)WM * 2 * BN * 4;
}
__host__ __device__ inline bool igemm_stage16(const ConvParams& p) {
  return !p.beta && !p.out_f32 && p.bias == nullptr && p.bnb_acc == nullptr;
}

// Output row of GEMM row m (strided-output remap: strided 1x1 data gradients, and the stride
// phases of a strided k x k data gradient, each phase one GEMM with its own origin).
__device__ __forceinline__ size_t epi_out_row(const ConvParams& p, int m) {
  if (!p.remap) return (size_t)m;
  const int PQ = p.P * p.Q;
  int n = m / PQ, r = m - n * PQ;
  int pp = r / p.Q, qq = r - pp * p.Q;
  return ((size_t)n * p.OH + (size_t)pp * p.osh + p.oh0) * p.OW + (size_t)qq * p.osw + p.ow0;
}

// remap == 2: a strided 1x1 data gradient that writes ALL of dx -- GEMM row m = (n, p, q) also
// stores zeros to the other pixels of its stride cell, (p*osh + a, q*osw + b) for (a, b) != (0, 0)
// (the host checks that the cells tile the output), so dx needs no zero-fill pass of its own
template <bool F32OUT>
__device__ __forceinline__ void epi_fill_cell(const ConvParams& p, int m, int col) {
  const int PQ = p.P * p.Q;
  const int n = m / PQ, r = m - n * PQ;
  const int pp = r / p.Q, qq = r - pp * p.Q;
  for (int a = 0; a < p.osh; ++a) {
    const int h = pp * p.osh + a;
    if (h >= p.OH) break;
    for (int b = (a == 0 ? 1 : 0); b < p.osw; ++b) {
      const int w = qq * p.osw + b;
      if (w >= p.OW) break;
      const size_t o = ((size_t)n * p.OH + h) * p.OW + w;
      if constexpr (F32OUT) {
        f32x4* yo = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.y) + o * p.ldy + col);
        yo[0] = f32x4{0.f, 0.f, 0.f, 0.f};
        yo[1] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        *reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(p.y) + o * p.ldy + col) = u32x4{0u, 0u, 0u, 0u};
      }
    }
  }
}

// Register prefetch of the fused BN-backward epilogue operands (z, y and the beta source) for
// one chunk of CH output segments per thread. A kernel with a short main loop issues the first
// chunk BEFORE its main loop, so these loads share one memory latency with the A/B tiles
// instead of paying a second one after the MFMAs (the stage-1 data-grad GEMMs have a single
// 64-deep k-step and are bound by exactly this latency).
// F32 (the fp32 path, conv_p3.hip): z, the beta source and the output g are fp32 (two 16-byte
// halves per 8-value segment: pr / pr2, pz / pz2), y is the bf16 hi plane of the activation
template <int WM, int WN, int TM, int TN, bool BNB, bool F32 = false>
struct EpiPrefetch {
  static constexpr int BM = WM * TM, BN = WN * TN, SEGS = BN / 8, NT = WM * WN * 64;
  static constexpr int ITER = BM * SEGS / NT;
  // (fp32: two segments per chunk -- its operands are twice the registers)
  static constexpr int CHMAX = F32 ? BNB_PREFETCH_CH / 2 : BNB_PREFETCH_CH;
  static constexpr int CH = BNB ? (ITER < CHMAX ? ITER : CHMAX) : 1;
  u32x4 pr[CH], pz[CH], py[CH];
  u32x4 pr2[F32 ? CH : 1], pz2[F32 ? CH : 1];
  // forward GEMMs: the BN statistic shift of each of the lane's accumulator columns, loaded
  // before the main loop so the epilogue does not wait on it
  static constexpr int NKC = BNB ? 1 : TN / 16;
  float kc[NKC];
  __device__ __forceinline__ void load_shift(const ConvParams& p, int n0, int wn, int lane) {
#pragma unroll
    for (int j = 0; j < NKC; ++j) {
      const int gcol = n0 + wn * TN + j * 16 + (lane & 15);
      kc[j] = (!BNB && p.stats != nullptr && p.stats_shift != nullptr && gcol < p.Nout) ? p.stats_shift[gcol] : 0.f;
    }
  }
  __device__ __forceinline__ void load(const ConvParams& p, int it0, int m0, int n0, int tid) {
    const int col = n0 + (tid % SEGS) * 8;
    if (col >= p.Nout) return;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int m = m0 + (tid + (it0 + k) * NT) / SEGS;
      if (m < p.M) {
        const size_t o = epi_out_row(p, m);
        if constexpr (F32) {
          if (p.beta) {
            const u32x4* r = reinterpret_cast<const u32x4*>(reinterpret_cast<const float*>(p.yres) + o * p.ldy + col);
            pr[k] = r[0];
            pr2[k] = r[1];
          }
          const u32x4* z = reinterpret_cast<const u32x4*>(reinterpret_cast<const float*>(p.bnb_z) + o * p.bnb_ld + col);
          pz[k] = z[0];
          pz2[k] = z[1];
        } else {
          if (p.beta)
            pr[k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(p.yres) + o * p.ldy + col);
          pz[k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(p.bnb_z) + o * p.bnb_ld + col);
        }
        if (p.bnb_mode == 1)
          py[k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(p.bnb_y) + o * p.bnb_ld + col);
      }
    }
  }
};

// Fused BN-backward: the tile's per-column (mean, invstd, gamma, beta) staged in LDS at kernel
// start (one float4 per column, above every other use of the workgroup's LDS), so the epilogue
// reads them with LDS latency instead of issuing 32 dependent global loads per thread after the
// MFMAs (a full memory round trip exposed per workgroup).
constexpr size_t bnb_param_lds(int BN) { return (size_t)BN * 16; }
template <int BN, int NT>
__device__ __forceinline__ void stage_bnb_params(const ConvParams& p, int n0, char* base) {
  float4* bp = reinterpret_cast<float4*>(base);
  for (int c = threadIdx.x; c < BN; c += NT) {
    const int gc = n0 + c;
    bp[c] = gc < p.Nout ? make_float4(p.bnb_mean[gc], p.bnb_invstd[gc], p.bnb_gamma[gc], p.bnb_beta[gc])
                        : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// In-launch split-K hand-off (cdna guide Guideline 16, counter form), shared by the LDS-DMA
// kernels: every split parks its partial tile in a workspace slab, publishes it with one
// agent-scope release + ticket; the last arriver acquires and sums ALL slabs in index order into
// acc and returns true (it then runs the epilogue), the others return false. Call after the main
// loop's final barrier (smem word 0 is used as the broadcast flag).
template <int MI, int NI, int NT>
__device__ __forceinline__ bool splitk_gather(const ConvParams& p, f32x4 (&acc)[MI][NI], char* smem, int tile,
                                              int split, int S, int tid) {
  constexpr int FR = MI * NI;  // f32x4 fragments per thread
  f32x4* slab = reinterpret_cast<f32x4*>(p.ws) + (size_t)tile * S * FR * NT;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) slab[((size_t)split * FR + i * NI + j) * NT + tid] = acc[i][j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(p.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == (unsigned)(S - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(p.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  const int last = *flag;
  __syncthreads();  // the flag word is epilogue staging space next
  if (!last) return false;
  // the sum in FIXED slab order 0..S-1 (the last arriver re-reads its own slab too): the fp32
  // result does not depend on which split arrived last, so split-K is run-to-run deterministic
  // (ADVICE r4); one extra slab read per tile
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = slab[((size_t)0 * FR + i * NI + j) * NT + tid];
  for (int s2 = 1; s2 < S; ++s2) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] += slab[((size_t)s2 * FR + i * NI + j) * NT + tid];
  }
  return true;
}

template <int WM, int WN, int TM, int TN, bool BNB, bool F32 = false>
__device__ __forceinline__ void igemm_epilogue(const ConvParams& p, f32x4 (&acc)[TM / 16][TN / 16], char* smem,
                                               int tm, int m0, int n0, int wm, int wn, int lane, int tid,
                                               EpiPrefetch<WM, WN, TM, TN, BNB, F32>& pre, bool prefetched,
                                               const char* bnb_params = nullptr) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int LDC = BN + 4;
  constexpr int SEGS = BN / 8;             // 16-byte output segments per tile row
  constexpr int NT = WM * WN * 64;         // threads of the workgroup
  constexpr int ITER = BM * SEGS / NT;     // segments per thread
  static_assert(NT % SEGS == 0 && ITER >= 1, "a thread keeps one column segment across the store pass");
  const int frow = lane & 15, fq = lane >> 4;
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC16 = BN + 8;  // 16-bit staging row (16-byte aligned rows)
  const bool s16 = !BNB && igemm_stage16(p);
  uint16_t* Cs16 = reinterpret_cast<uint16_t*>(smem);
  float* red = s16 ? reinterpret_cast<float*>(smem + (size_t)BM * LDC16 * 2)
                   : Cs + BM * LDC;  // [WM][2][BN] per-wave column partial sums
  if (p.stats != nullptr) {
    // per-column partial BN statistics straight from the accumulators, shifted by the
    // column's K: sum the wave's row quads in registers, then across the 4 lane groups that
    // share a column with two xor-shuffles. Rows at or beyond M (only in the last row tile)
    // are skipped: their zero accumulators would otherwise add (-K)^2.
    const int wrows = p.M - (m0 + wm * TM);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      float s1 = 0.f, s2 = 0.f;
      float kc = 0.f;
      if constexpr (!BNB) kc = pre.kc[j];
      if (wrows >= TM) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = acc[i][j][e] - kc;
            s1 += v;
            s2 += v * v;
          }
      } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = i * 16 + fq * 4 + e < wrows ? acc[i][j][e] - kc : 0.f;
            s1 += v;
            s2 += v * v;
          }
      }
      s1 += __shfl_xor(s1, 16, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (fq == 0) {
        red[(wm * 2) * BN + wn * TN + j * 16 + frow] = s1;
        red[(wm * 2 + 1) * BN + wn * TN + j * 16 + frow] = s2;
      }
    }
  }
  if (s16) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int row = wm * TM + i * 16 + fq * 4 + e;
          int col = wn * TN + j * 16 + frow;
          Cs16[row * LDC16 + col] = f2act(acc[i][j][e]);
        }
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int row = wm * TM + i * 16 + fq * 4 + e;
          int col = wn * TN + j * 16 + frow;
          Cs[row * LDC + col] = acc[i][j][e];
        }
  }

  const int cs = tid % SEGS;
  const int col = n0 + cs * 8;
  const bool col_ok = col < p.Nout;
  const int PQ = p.P * p.Q;
  auto out_row = [&](int m) -> size_t { return epi_out_row(p, m); };
  auto load_seg = [](const void* base, size_t row, int ld, int c) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(base) + row * ld + c);
  };
  (void)PQ;

  // fused BN-backward: the first chunk of z / y / beta-source segments is in flight before
  // the barrier (or since before the main loop); registers hold one chunk
  constexpr int CH = EpiPrefetch<WM, WN, TM, TN, BNB, F32>::CH;
  if constexpr (BNB) {
    if (!prefetched) pre.load(p, 0, m0, n0, tid);
  }
  __syncthreads();

  if (p.stats != nullptr) {
    for (int c = tid; c < BN; c += NT) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s1 += red[(w * 2) * BN + c];
        s2 += red[(w * 2 + 1) * BN + c];
      }
      int gc = n0 + c;
      if (gc < p.Nout) {
        if (p.stats_R > 0) {  // atomics into replica tm % R of a [R][2][Nout] accumulator
          float* dst = p.stats + (size_t)(tm % p.stats_R) * 2 * p.Nout;
          atomicAdd(dst + gc, s1);
          atomicAdd(dst + p.Nout + gc, s2);
        } else {
          p.stats[(size_t)tm * 2 * p.Nout + gc] = s1;
          p.stats[(size_t)tm * 2 * p.Nout + p.Nout + gc] = s2;
        }
      }
    }
  }

  auto stage_row = [&](int row, float* v) {
    const f32x4* src = reinterpret_cast<const f32x4*>(Cs + row * LDC + cs * 8);
    f32x4 v0 = src[0], v1 = src[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = v0[e];
      v[4 + e] = v1[e];
    }
  };

  if constexpr (!BNB) {
    if (s16) {  // bf16 output, no beta / bias: rows of 8 staged 16-bit values, optional ReLU
      for (int it = 0; it < ITER; ++it) {
        const int row = (tid + it * NT) / SEGS;
        const int m = m0 + row;
        if (!col_ok || m >= p.M) continue;
        u32x4 v = *reinterpret_cast<const u32x4*>(Cs16 + row * LDC16 + cs * 8);
        if (p.relu) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
          v = pack8(f);
        }
        *reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(p.y) + out_row(m) * p.ldy + col) = v;
        if (p.remap == 2) epi_fill_cell<false>(p, m, col);
      }
      return;
    }
    for (int it = 0; it < ITER; ++it) {
      const int row = (tid + it * NT) / SEGS;
      const int m = m0 + row;
      if (!col_ok || m >= p.M) continue;
      const size_t orow = out_row(m);
      float v[8];
      stage_row(row, v);
      if (p.bias != nullptr) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (col + e < p.Nout) ? p.bias[col + e] : 0.f;
      }
      if (p.relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (p.out_f32) {
        float* yo = reinterpret_cast<float*>(p.y) + orow * p.ldy + col;
        if (p.beta) {
          const float* yi = reinterpret_cast<const float*>(p.yres) + orow * p.ldy + col;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += yi[e];
        }
        reinterpret_cast<f32x4*>(yo)[0] = f32x4{v[0], v[1], v[2], v[3]};
        reinterpret_cast<f32x4*>(yo)[1] = f32x4{v[4], v[5], v[6], v[7]};
        if (p.remap == 2) epi_fill_cell<true>(p, m, col);
      } else {
        uint16_t* yo = reinterpret_cast<uint16_t*>(p.y) + orow * p.ldy + col;
        if (p.beta) {
          float o[8];
          unpack8(load_seg(p.yres, orow, p.ldy, col), o);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += o[e];
        }
        *reinterpret_cast<u32x4*>(yo) = pack8(v);
        if (p.remap == 2) epi_fill_cell<false>(p, m, col);
      }
    }
  } else {
    // 16-bit (fp32 on the F32 path) output, no bias / relu (checked on the host)
    float bmu[8], bis[8], bsc[8], bsh[8], bs1[8], bs2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool okc = col + e < p.Nout;
      if (bnb_params != nullptr) {
        const float4 q = reinterpret_cast<const float4*>(bnb_params)[cs * 8 + e];  // zeros past Nout
        bmu[e] = q.x;
        bis[e] = q.y;
        bsc[e] = q.z * q.y;
        bsh[e] = q.w - q.x * bsc[e];
      } else {  // the LDS budget had no room (deepest rings): global loads
        bmu[e] = okc ? p.bnb_mean[col + e] : 0.f;
        bis[e] = okc ? p.bnb_invstd[col + e] : 0.f;
        bsc[e] = okc ? p.bnb_gamma[col + e] * bis[e] : 0.f;
        bsh[e] = okc ? p.bnb_beta[col + e] - bmu[e] * bsc[e] : 0.f;
      }
      bs1[e] = 0.f;
      bs2[e] = 0.f;
    }
    for (int it0 = 0; it0 < ITER; it0 += CH) {
      if (it0 > 0) pre.load(p, it0, m0, n0, tid);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int row = (tid + (it0 + k) * NT) / SEGS;
        const int m = m0 + row;
        if (!col_ok || m >= p.M) continue;
        const size_t orow = out_row(m);
        float v[8];
        stage_row(row, v);
        auto f32x8 = [](const u32x4& a, const u32x4& b, float* f) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            f[e] = __uint_as_float(a[e]);
            f[4 + e] = __uint_as_float(b[e]);
          }
        };
        if (p.beta) {
          float o[8];
          if constexpr (F32)
            f32x8(pre.pr[k], pre.pr2[k], o);
          else
            unpack8(pre.pr[k], o);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += o[e];
        }
        float zf[8];
        if constexpr (F32)
          f32x8(pre.pz[k], pre.pz2[k], zf);
        else
          unpack8(pre.pz[k], zf);
        if (p.bnb_mode == 1) {
          float yf[8];
          if constexpr (F32)
            unpack_bf16x8(pre.py[k], yf);  // the hi plane: > 0 exactly when y > 0
          else
            unpack8(pre.py[k], yf);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = yf[e] > 0.f ? v[e] : 0.f;
        } else if (p.bnb_mode == 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (zf[e] * bsc[e] + bsh[e]) > 0.f ? v[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bs1[e] += v[e];
          bs2[e] += v[e] * ((zf[e] - bmu[e]) * bis[e]);
        }
        if constexpr (F32) {
          f32x4* yo = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.y) + orow * p.ldy + col);
          yo[0] = f32x4{v[0], v[1], v[2], v[3]};
          yo[1] = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          *reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(p.y) + orow * p.ldy + col) = pack8(v);
        }
        if (p.remap == 2) epi_fill_cell<F32>(p, m, col);
      }
    }
    // threads sharing a column segment: LDS partials [NT/SEGS][BN] (x2), column sums, atomics
    constexpr int PR = NT / SEGS;
    static_assert(2 * PR * BN <= BM * LDC, "partials fit in the staging buffer");
    float* part = Cs;
    __syncthreads();  // all Cs reads of the store pass are done
    const int r = tid / SEGS;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      part[r * BN + cs * 8 + e] = bs1[e];
      part[PR * BN + r * BN + cs * 8 + e] = bs2[e];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float a = 0.f, b = 0.f;
#pragma unroll 4
      for (int rr = 0; rr < PR; ++rr) {
        a += part[rr * BN + c];
        b += part[PR * BN + rr * BN + c];
      }
      const int gc = n0 + c;
      if (gc < p.Nout) {
        float* dst = p.bnb_acc + (size_t)(tm % p.bnb_R) * 2 * p.Nout;
        atomicAdd(dst + gc, a);
        atomicAdd(dst + p.Nout + gc, b);
      }
    }
  }
}

}  // namespace hcb
