// Training-mode batch normalisation for NHWC bf16 activations on gfx950
// (the MKL-DNN FusedBatchNorm fwd/bwd role; tf_cnn_benchmarks ResNet
// config decay=0.9, eps=1e-5, scale=True).
//
// Layout: x is [M = N*H*W][C] with C contiguous. Every thread owns one 16-byte vector of
// 8 channels, keeps that channel vector's scale/shift (or partial sums) in registers and
// walks rows, so every global access is a 16-byte coalesced load/store and the per
// channel parameters are read once per thread (guide: always vectorize bf16).
//
// Statistics are reduced in two levels: per-block partial sums in an fp32 slab
// [T][2][C] (the conv epilogue writes the same slab format, so stats can be fused into
// the producing GEMM), then a finalize kernel that sums the slab in fp64 — no float
// atomics, bitwise reproducible.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace hcb {

constexpr int BN_U = 4;  // rows in flight per thread in the streaming kernels
constexpr int BN_UB = 2;  // the backward reduce / apply: 2 rows (x 3 tensors) in flight -- 119 VGPRs, occupancy 4,
                          // against 151 / 3 at 4 rows (+18% on the mid-size tensors, profiles/r4bn_rows_ab.txt)

// buffer-resource byte range covering rows [0, M) of a [M][ld] bf16 tensor (clamped to 2 GiB)
__device__ __forceinline__ uint32_t rsrc_bytes(int M, int ld, int esz = 2) {
  size_t b = (size_t)M * (size_t)ld * (size_t)esz;
  return b > 0x7fffffffu ? 0x7fffffffu : (uint32_t)b;
}

// thread -> (channel vector, row lane) mapping shared by all kernels below
struct RowMap {
  int cv, r0, rstep, active;
};
__device__ __forceinline__ RowMap rowmap(int C) {
  RowMap m;
  int CV = C >> 3;
  int rows = 256 / CV;
  m.cv = threadIdx.x % CV;
  m.r0 = threadIdx.x / CV;
  m.rstep = rows;
  m.active = m.r0 < rows;
  return m;
}

// reduce per-thread partial (s1, s2) over threads sharing a channel vector, write slab row
__device__ __forceinline__ void slab_write(float* lds, const float* s1, const float* s2, int C,
                                           const RowMap& rm, float* slab_row) {
  int CV = C >> 3;
  int rows = 256 / CV;
  // lds: [rows][C] for s1 then s2
  if (rm.active) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lds[rm.r0 * C + rm.cv * 8 + e] = s1[e];
      lds[rows * C + rm.r0 * C + rm.cv * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rows; ++r) {
      a += lds[r * C + c];
      b += lds[rows * C + r * C + c];
    }
    slab_row[c] = a;
    slab_row[C + c] = b;
  }
}

__global__ __launch_bounds__(256) void bn_stats_kernel(const uint16_t* __restrict__ x, int M, int C,
                                                       int ldx, float* slab) {
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  RowMap rm = rowmap(C);
  float s1[8] = {0}, s2[8] = {0};
  if (rm.active) {
    for (int m = blockIdx.x * rm.rstep + rm.r0; m < M; m += gridDim.x * rm.rstep) {
      u32x4 v = *reinterpret_cast<const u32x4*>(x + (size_t)m * ldx + rm.cv * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += f[e];
        s2[e] += f[e] * f[e];
      }
    }
  }
  slab_write(lds_f, s1, s2, C, rm, slab + (size_t)blockIdx.x * 2 * C);
}

// Parallel slab reduction: a block owns 64 channels (one per lane, so every load is a
// 256-byte coalesced row segment); its 8 waves stride over the T partial rows with 4
// independent loads in flight each, accumulate in fp64, then combine through LDS.
constexpr int FIN_WAVES = 8;
__device__ __forceinline__ void slab_reduce64(const float* slab, int T, int C, double* a_out,
                                              double* b_out, double* lds) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double a = 0.0, b = 0.0;
  if (c < C) {
    int t = wid;
    for (; t + 3 * FIN_WAVES < T; t += 4 * FIN_WAVES) {
      float x0 = slab[(size_t)t * 2 * C + c], y0 = slab[(size_t)t * 2 * C + C + c];
      float x1 = slab[(size_t)(t + FIN_WAVES) * 2 * C + c], y1 = slab[(size_t)(t + FIN_WAVES) * 2 * C + C + c];
      float x2 = slab[(size_t)(t + 2 * FIN_WAVES) * 2 * C + c],
            y2 = slab[(size_t)(t + 2 * FIN_WAVES) * 2 * C + C + c];
      float x3 = slab[(size_t)(t + 3 * FIN_WAVES) * 2 * C + c],
            y3 = slab[(size_t)(t + 3 * FIN_WAVES) * 2 * C + C + c];
      a += ((double)x0 + (double)x1) + ((double)x2 + (double)x3);
      b += ((double)y0 + (double)y1) + ((double)y2 + (double)y3);
    }
    for (; t < T; t += FIN_WAVES) {
      a += (double)slab[(size_t)t * 2 * C + c];
      b += (double)slab[(size_t)t * 2 * C + C + c];
    }
  }
  lds[wid * 64 + lane] = a;
  lds[FIN_WAVES * 64 + wid * 64 + lane] = b;
  __syncthreads();
  if (wid == 0) {
    a = 0.0;
    b = 0.0;
#pragma unroll
    for (int w = 0; w < FIN_WAVES; ++w) {
      a += lds[w * 64 + lane];
      b += lds[FIN_WAVES * 64 + w * 64 + lane];
    }
  }
  *a_out = a;
  *b_out = b;
}

__global__ __launch_bounds__(512) void bn_finalize_kernel(const float* slab, int T, int C, double count,
                                                          float eps, float momentum, float* mean,
                                                          float* invstd, float* run_mean,
                                                          float* run_var) {
  __shared__ double lds[2 * FIN_WAVES * 64];
  double a, b;
  slab_reduce64(slab, T, C, &a, &b, lds);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  double mu = a / count;
  double var = b / count - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean != nullptr) {
    double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    run_mean[c] = (float)(momentum * run_mean[c] + (1.0 - momentum) * mu);
    run_var[c] = (float)(momentum * run_var[c] + (1.0 - momentum) * unbiased);
  }
}

__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ x, int ldx,
                                                       uint16_t* __restrict__ y, int ldy,
                                                       const uint16_t* __restrict__ res, int ldr,
                                                       int M, int C, const float* mean,
                                                       const float* invstd, const float* gamma,
                                                       const float* beta, int relu) {
  RowMap rm = rowmap(C);
  if (!rm.active) return;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    int c = rm.cv * 8 + e;
    float s = gamma[c] * invstd[c];
    sc[e] = s;
    sh[e] = beta[c] - mean[c] * s;
  }
  // BN_U rows in flight per thread: every load of the group is issued before any use
  // (buffer loads, out-of-range rows return zeros -> no branches around loads)
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, rsrc_bytes(M, ldx));
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(res != nullptr ? res : x, rsrc_bytes(M, res != nullptr ? ldr : ldx));
  const int stride = gridDim.x * rm.rstep;
  for (int m0 = blockIdx.x * rm.rstep + rm.r0; m0 < M; m0 += BN_U * stride) {
    u32x4 xv[BN_U], rv[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      int m = m0 + u * stride;
      xv[u] = buf_load16(xr, m < M ? (uint32_t)((size_t)m * ldx + rm.cv * 8) * 2u : HCB_OOB);
      if (res != nullptr) rv[u] = buf_load16(rr, m < M ? (uint32_t)((size_t)m * ldr + rm.cv * 8) * 2u : HCB_OOB);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      int m = m0 + u * stride;
      float f[8];
      unpack8(xv[u], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = f[e] * sc[e] + sh[e];
      if (res != nullptr) {
        float r[8];
        unpack8(rv[u], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += r[e];
      }
      if (relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
      }
      if (m < M) *reinterpret_cast<u32x4*>(y + (size_t)m * ldy + rm.cv * 8) = pack8(f);
    }
  }
}

// relu: 0 = none, 1 = mask from stored output y (y > 0), 2 = mask recomputed from x
// (gamma*xhat + beta > 0; valid when the block had no residual add)
struct BwdSrc {
  __amdgpu_buffer_rsrc_t dyr, xr, yr;
  int lddy, ldx, ldyv, cv;
  __device__ __forceinline__ void load(int m, int M, int relu, u32x4& d, u32x4& x, u32x4& y) const {
    const bool ok = m < M;
    d = buf_load16(dyr, ok ? (uint32_t)((size_t)m * lddy + cv * 8) * 2u : HCB_OOB);
    x = buf_load16(xr, ok ? (uint32_t)((size_t)m * ldx + cv * 8) * 2u : HCB_OOB);
    if (relu == 1) y = buf_load16(yr, ok ? (uint32_t)((size_t)m * ldyv + cv * 8) * 2u : HCB_OOB);
  }
};
__device__ __forceinline__ void bwd_math(const u32x4& dv, const u32x4& xvv, const u32x4& yvv, int relu,
                                         const float* mu, const float* is, const float* sc, const float* sh,
                                         float* g, float* xh) {
  float d[8], xv[8];
  unpack8(dv, d);
  unpack8(xvv, xv);
#pragma unroll
  for (int e = 0; e < 8; ++e) xh[e] = (xv[e] - mu[e]) * is[e];
  if (relu == 1) {
    float yv[8];
    unpack8(yvv, yv);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = yv[e] > 0.f ? d[e] : 0.f;
  } else if (relu == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = (xv[e] * sc[e] + sh[e]) > 0.f ? d[e] : 0.f;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = d[e];
  }
}

// element-type generic forms (T = the build's 16-bit type or fp32) used by the finalize-free kernels
// TY: element type of the ReLU-mask source y -- T, or (fp32 path) uint16_t: the bf16 hi plane of the
// plane-stored activation (hi > 0 exactly when y > 0 for every normal y)
// BN backward fed straight from a max-pool's gradient (the ResNet stem: BN -> ReLU -> 3x3/2 max
// pool): dy of pixel (n, h, w) is gathered from the pooled gradient dyp of the <= 2x2 windows that
// contain it and whose argmax (amax, window-local index per channel) is this pixel -- the
// full-size dy is never written (it was written by maxpool_bwd_amax_kernel and read twice).
template <typename T>
__device__ __forceinline__ void pool_gather(const PoolSrc& ps, int m, int M, int cv, Act8<T>& d) {
  float g[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = 0.f;
  if (m < M) {
    const int w = m % ps.W, t = m / ps.W;
    const int h = t % ps.H, n = t / ps.H;
    const int p_hi = (h + ps.pt) / ps.s, q_hi = (w + ps.pl) / ps.s;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = p_hi - i;
      if (p < 0 || p >= ps.P || h - (p * ps.s - ps.pt) >= ps.k) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = q_hi - j;
        if (q < 0 || q >= ps.Q || w - (q * ps.s - ps.pl) >= ps.k) continue;
        const size_t o = (size_t)(n * ps.P + p) * ps.Q + q;
        const int mine = (h - (p * ps.s - ps.pt)) * ps.k + (w - (q * ps.s - ps.pl));
        const u32x2 a = *reinterpret_cast<const u32x2*>(ps.amax + o * ps.C + cv * 8);
        Act8<T> dv;
        dv.load(reinterpret_cast<const T*>(ps.dyp) + o * ps.ldp + cv * 8);
        float f[8];
        dv.to_f(f);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((int)((a[e >> 2] >> (8 * (e & 3))) & 0xff) == mine) g[e] += f[e];
      }
    }
  }
  d.set_f(g);
}

template <typename T, typename TY = T, bool POOL = false>
struct BwdSrcT {
  __amdgpu_buffer_rsrc_t dyr, xr, yr;
  int lddy, ldx, ldyv, cv;
  PoolSrc pool;
  __device__ __forceinline__ void load(int m, int M, int relu, Act8<T>& d, Act8<T>& x, Act8<TY>& y) const {
    const bool ok = m < M;
    constexpr uint32_t E = Act8<T>::ESZ;
    if constexpr (POOL)
      pool_gather<T>(pool, m, M, cv, d);
    else
      d.load(dyr, ok ? (uint32_t)((size_t)m * lddy + cv * 8) * E : HCB_OOB);
    x.load(xr, ok ? (uint32_t)((size_t)m * ldx + cv * 8) * E : HCB_OOB);
    if (relu == 1) y.load(yr, ok ? (uint32_t)((size_t)m * ldyv + cv * 8) * Act8<TY>::ESZ : HCB_OOB);
  }
};
template <typename T, typename TY = T>
__device__ __forceinline__ void bwd_math_t(const Act8<T>& dv, const Act8<T>& xvv, const Act8<TY>& yvv, int relu,
                                           const float* mu, const float* is, const float* sc, const float* sh,
                                           float* g, float* xh) {
  float d[8], xv[8];
  dv.to_f(d);
  xvv.to_f(xv);
#pragma unroll
  for (int e = 0; e < 8; ++e) xh[e] = (xv[e] - mu[e]) * is[e];
  if (relu == 1) {
    float yv[8];
    yvv.to_f(yv);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = yv[e] > 0.f ? d[e] : 0.f;
  } else if (relu == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = (xv[e] * sc[e] + sh[e]) > 0.f ? d[e] : 0.f;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = d[e];
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const uint16_t* __restrict__ dy, int lddy, const uint16_t* __restrict__ y, int ldyv,
    const uint16_t* __restrict__ x, int ldx, int M, int C, const float* mean, const float* invstd,
    const float* gamma, const float* beta, int relu, float* slab, uint16_t* gout, int ldg) {
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  RowMap rm = rowmap(C);
  float s1[8] = {0}, s2[8] = {0};
  if (rm.active) {
    float mu[8], is[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int c = rm.cv * 8 + e;
      mu[e] = mean[c];
      is[e] = invstd[c];
      sc[e] = gamma != nullptr ? gamma[c] * is[e] : 0.f;
      sh[e] = beta != nullptr ? beta[c] - mu[e] * sc[e] : 0.f;
    }
    BwdSrc src{make_rsrc(dy, rsrc_bytes(M, lddy)), make_rsrc(x, rsrc_bytes(M, ldx)),
               make_rsrc(y != nullptr ? y : x, rsrc_bytes(M, y != nullptr ? ldyv : ldx)), lddy, ldx, ldyv, rm.cv};
    const int stride = gridDim.x * rm.rstep;
    for (int m0 = blockIdx.x * rm.rstep + rm.r0; m0 < M; m0 += BN_U * stride) {
      u32x4 dv[BN_U], xv[BN_U], yv[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) src.load(m0 + u * stride, M, relu, dv[u], xv[u], yv[u]);
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const int m = m0 + u * stride;
        float g[8], xh[8];
        bwd_math(dv[u], xv[u], yv[u], relu, mu, is, sc, sh, g, xh);
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // rows beyond M load zeros: g = 0 contributes nothing
          s1[e] += g[e];
          s2[e] += g[e] * xh[e];
        }
        if (gout != nullptr && m < M) *reinterpret_cast<u32x4*>(gout + (size_t)m * ldg + rm.cv * 8) = pack8(g);
      }
    }
  }
  slab_write(lds_f, s1, s2, C, rm, slab + (size_t)blockIdx.x * 2 * C);
}

__global__ __launch_bounds__(512) void bn_bwd_finalize_kernel(const float* slab, int T, int C,
                                                              float* dgamma, float* dbeta) {
  __shared__ double lds[2 * FIN_WAVES * 64];
  double a, b;
  slab_reduce64(slab, T, C, &a, &b, lds);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  dbeta[c] = (float)a;
  dgamma[c] = (float)b;
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const uint16_t* __restrict__ dy, int lddy, const uint16_t* __restrict__ y, int ldyv,
    const uint16_t* __restrict__ x, int ldx, uint16_t* __restrict__ dx, int lddx, int M, int C,
    const float* mean, const float* invstd, const float* gamma, const float* beta,
    const float* dgamma, const float* dbeta, int relu) {
  RowMap rm = rowmap(C);
  if (!rm.active) return;
  float mu[8], is[8], sc[8], sh[8], k1[8], k2[8];
  const float invM = 1.f / (float)M;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    int c = rm.cv * 8 + e;
    mu[e] = mean[c];
    is[e] = invstd[c];
    sc[e] = gamma[c] * is[e];
    sh[e] = beta[c] - mu[e] * sc[e];
    k1[e] = dbeta[c] * invM;
    k2[e] = dgamma[c] * invM;
  }
  BwdSrc src{make_rsrc(dy, rsrc_bytes(M, lddy)), make_rsrc(x, rsrc_bytes(M, ldx)),
             make_rsrc(y != nullptr ? y : x, rsrc_bytes(M, y != nullptr ? ldyv : ldx)), lddy, ldx, ldyv, rm.cv};
  const int stride = gridDim.x * rm.rstep;
  for (int m0 = blockIdx.x * rm.rstep + rm.r0; m0 < M; m0 += BN_U * stride) {
    u32x4 dv[BN_U], xv[BN_U], yv[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) src.load(m0 + u * stride, M, relu, dv[u], xv[u], yv[u]);
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const int m = m0 + u * stride;
      float g[8], xh[8], o[8];
      bwd_math(dv[u], xv[u], yv[u], relu, mu, is, sc, sh, g, xh);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = sc[e] * (g[e] - k1[e] - xh[e] * k2[e]);
      if (m < M) *reinterpret_cast<u32x4*>(dx + (size_t)m * lddx + rm.cv * 8) = pack8(o);
    }
  }
}

static int bn_grid(int M, int C) {
  int rows = 256 / (C / 8);
  int need = (M + rows - 1) / rows;
  // ~4 blocks per CU over 256 CUs; each block loops over its rows
  int g = need < 1024 ? need : 1024;
  return g < 1 ? 1 : g;
}

int bn_num_partials(int M, int C) { return bn_grid(M, C); }

// ---------------------------------------------------------------------------------------
// One-launch two-level finalize. Grid (C/64 channel groups) x (S row splits): each block
// reduces T/S slab rows for 64 channels (fp64) into part[S][2][C]; the LAST block of a
// channel group (agent-scope release -> ticket atomic -> acquire, the placement-independent
// hand-off of the CDNA guide, Guideline 16) sums the S partials and writes the outputs, then
// re-arms its counter. Counters start zeroed at module load and are left zeroed by every
// launch, so graph replays need no memset.
__device__ unsigned g_fin_counters[64];

template <bool FWD>
__global__ __launch_bounds__(512) void bn_finalize_split_kernel(
    const float* __restrict__ slab, int T, int C, int rows_per, double* part, double count, float eps,
    float momentum, float* mean, float* invstd, float* run_mean, float* run_var, float* dgamma,
    float* dbeta) {
  __shared__ double lds[2 * FIN_WAVES * 64];
  __shared__ int last;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int S = gridDim.y;
  const int t0 = blockIdx.y * rows_per;
  const int t1 = min(T, t0 + rows_per);
  double a = 0.0, b = 0.0;
  if (c < C) {
    for (int t = t0 + wid; t < t1; t += FIN_WAVES) {
      a += (double)slab[(size_t)t * 2 * C + c];
      b += (double)slab[(size_t)t * 2 * C + C + c];
    }
  }
  lds[wid * 64 + lane] = a;
  lds[FIN_WAVES * 64 + wid * 64 + lane] = b;
  __syncthreads();
  if (wid == 0 && c < C) {
    a = 0.0;
    b = 0.0;
#pragma unroll
    for (int w = 0; w < FIN_WAVES; ++w) {
      a += lds[w * 64 + lane];
      b += lds[FIN_WAVES * 64 + w * 64 + lane];
    }
    part[(size_t)blockIdx.y * 2 * C + c] = a;
    part[(size_t)blockIdx.y * 2 * C + C + c] = b;
  }
  // publish: every storing wave drains, barrier, one release + ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned tk = __hip_atomic_fetch_add(&g_fin_counters[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    last = (tk == (unsigned)(S - 1));
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (wid != 0) return;
  if (c < C) {
    a = 0.0;
    b = 0.0;
    for (int s = 0; s < S; ++s) {
      a += part[(size_t)s * 2 * C + c];
      b += part[(size_t)s * 2 * C + C + c];
    }
    if constexpr (FWD) {
      double mu = a / count;
      double var = b / count - mu * mu;
      if (var < 0.0) var = 0.0;
      mean[c] = (float)mu;
      invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
      if (run_mean != nullptr) {
        double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
        run_mean[c] = (float)(momentum * run_mean[c] + (1.0 - momentum) * mu);
        run_var[c] = (float)(momentum * run_var[c] + (1.0 - momentum) * unbiased);
      }
    } else {
      dbeta[c] = (float)a;
      dgamma[c] = (float)b;
    }
  }
  if (lane == 0) __hip_atomic_store(&g_fin_counters[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int bn_finalize_splits(int T) {
  int s = (T + 63) / 64;
  return s < 1 ? 1 : (s > 32 ? 32 : s);
}

void launch_bn_finalize_split(const float* slab, int T, int C, double* part, int fwd, double count, float eps,
                              float momentum, float* mean, float* invstd, float* run_mean, float* run_var,
                              float* dgamma, float* dbeta, hipStream_t st) {
  int S = bn_finalize_splits(T);
  int rows_per = (T + S - 1) / S;
  S = (T + rows_per - 1) / rows_per;
  dim3 grid((C + 63) / 64, S);
  if (fwd)
    hipLaunchKernelGGL(bn_finalize_split_kernel<true>, grid, dim3(64 * FIN_WAVES), 0, st, slab, T, C, rows_per,
                       part, count, eps, momentum, mean, invstd, run_mean, run_var, nullptr, nullptr);
  else
    hipLaunchKernelGGL(bn_finalize_split_kernel<false>, grid, dim3(64 * FIN_WAVES), 0, st, slab, T, C, rows_per,
                       part, 0.0, 0.f, 0.f, nullptr, nullptr, nullptr, nullptr, dgamma, dbeta);
}

void launch_bn_stats(const void* x, int M, int C, int ldx, float* slab, int T, hipStream_t st) {
  int rows = 256 / (C / 8);
  size_t lds = (size_t)2 * rows * C * 4;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(T), dim3(256), lds, st, (const uint16_t*)x, M, C, ldx,
                     slab);
}

void launch_bn_finalize(const float* slab, int T, int C, double count, float eps, float momentum,
                        float* mean, float* invstd, float* run_mean, float* run_var,
                        hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, st, slab, T, C,
                     count, eps, momentum, mean, invstd, run_mean, run_var);
}

void launch_bn_apply(const void* x, int ldx, void* y, int ldy, const void* res, int ldr, int M,
                     int C, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, int relu, hipStream_t st) {
  hipLaunchKernelGGL(bn_apply_kernel, dim3(bn_grid(M, C)), dim3(256), 0, st, (const uint16_t*)x,
                     ldx, (uint16_t*)y, ldy, (const uint16_t*)res, ldr, M, C, mean, invstd, gamma,
                     beta, relu);
}

void launch_bn_bwd_reduce2(const void* dy, int lddy, const void* y, int ldyv, const void* x,
                           int ldx, int M, int C, const float* mean, const float* invstd,
                           const float* gamma, const float* beta, int relu, float* slab, int T,
                           void* gout, int ldg, hipStream_t st) {
  int rows = 256 / (C / 8);
  size_t lds = (size_t)2 * rows * C * 4;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(T), dim3(256), lds, st, (const uint16_t*)dy, lddy,
                     (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx, M, C, mean, invstd, gamma,
                     beta, relu, slab, (uint16_t*)gout, ldg);
}

void launch_bn_bwd_finalize(const float* slab, int T, int C, float* dgamma, float* dbeta,
                            hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, st, slab, T, C,
                     dgamma, dbeta);
}

void launch_bn_bwd_apply2(const void* dy, int lddy, const void* y, int ldyv, const void* x, int ldx,
                          void* dx, int lddx, int M, int C, const float* mean, const float* invstd,
                          const float* gamma, const float* beta, const float* dgamma,
                          const float* dbeta, int relu, hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(bn_grid(M, C)), dim3(256), 0, st,
                     (const uint16_t*)dy, lddy, (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx,
                     (uint16_t*)dx, lddx, M, C, mean, invstd, gamma, beta, dgamma, dbeta, relu);
}

}  // namespace hcb


// =======================================================================================
// Finalize-free BN: statistics are accumulated with fp32 atomics into R replicas of a
// [2][C] accumulator (producer tile t adds into replica t % R, spreading the contention);
// the consumer kernel reduces the replicas itself and derives mean/invstd (or dgamma/dbeta),
// which removes the separate finalize launch per BN layer (two per layer per step).
// Accumulators are zeroed once per step by one memset.
//
// Blocks tile (row split) x (channel group of CB = 8*CVB channels): a block reduces only
// its group's R*2*CB replica floats (4 KiB for CB = 64) instead of all C channels, and a
// row segment of a group is CB*2 = 128 contiguous bytes, so loads stay line-sized.
// =======================================================================================
namespace hcb {

// channel vectors (of 8) per group: 8 when possible, else the whole (small) C, else the
// largest divisor <= 32
static int bn_group_vecs(int CV) {
  if (CV % 8 == 0) return 8;
  if (CV <= 32) return CV;
  for (int d = 32; d > 1; --d)
    if (CV % d == 0) return d;
  return 1;
}

struct GroupMap {
  int cv, r0, rows, c0, CB;
};
__device__ __forceinline__ GroupMap groupmap(int CVB) {
  GroupMap g;
  g.CB = CVB * 8;
  g.c0 = blockIdx.y * g.CB;
  g.rows = 256 / CVB;
  g.r0 = threadIdx.x / CVB;
  g.cv = blockIdx.y * CVB + (threadIdx.x % CVB);
  return g;
}

// channel c's two replica sums (R replicas of [2][C]). R8 (the STAT_R = 8 training case): straight-
// line loads, so the whole coefficient body is one block whose loads issue in one round trip (a
// runtime replica loop let the compiler hoist the parameter math above it: two round trips)
template <bool R8>
__device__ __forceinline__ void sum_replicas2(const float* __restrict__ acc, int R, int C, int c, float& s, float& q) {
  s = 0.f;
  q = 0.f;
  if constexpr (R8) {
    float a[8], b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a[r] = acc[(size_t)r * 2 * C + c];
      b[r] = acc[(size_t)r * 2 * C + C + c];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      s += a[r];
      q += b[r];
    }
  } else {
    for (int r = 0; r < R; ++r) {
      s += acc[(size_t)r * 2 * C + c];
      q += acc[(size_t)r * 2 * C + C + c];
    }
  }
}
template <bool R8>
__device__ __forceinline__ void bn_coef_fwd(const float* __restrict__ acc, int R, int C, int c0, int CB, int M,
                                            float eps, float momentum, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, const float* __restrict__ K, bool publish,
                                            float* smean, float* sinv, float* rmean, float* rvar, float* coef,
                                            int i0, int step) {
  const float inv_n = 1.f / (float)M;
  for (int i = i0; i < CB; i += step) {
    const int c = c0 + i;
    float s, q;
    sum_replicas2<R8>(acc, R, C, c, s, q);
    const float g = gamma[c], bt = beta[c], k = K != nullptr ? K[c] : 0.f;
    const float d = s * inv_n;  // E[v - K]
    const float mu = d + k;
    const float var = fmaxf(q * inv_n - d * d, 0.f);
    const float is = rsqrtf(var + eps);
    const float sc = g * is;
    coef[i] = sc;
    coef[CB + i] = bt - mu * sc;
    if (publish) {
      smean[c] = mu;
      sinv[c] = is;
      if (rmean != nullptr) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        rmean[c] = momentum * rmean[c] + (1.f - momentum) * mu;
        rvar[c] = momentum * rvar[c] + (1.f - momentum) * unb;
      }
    }
  }
}
// 8 consecutive floats of an LDS table (16-byte aligned) into registers
__device__ __forceinline__ void lds_read8(const float* p, float* o) {
  const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o[e] = a[e];
    o[4 + e] = b[e];
  }
}

// RBN: the residual operand is a projection shortcut's raw conv output normalised here (ResBN);
// its own instantiation, so the common kernel keeps its register budget
// P3 (fp32 path): y is written as bf16 hi / mid / lo planes (plane stride yps elements) -- the
// GEMM-operand format of the consuming convs -- and a plain residual (!RBN, the identity shortcut:
// the block input) is read from its planes (plane stride rps); T = float (z, and an RBN residual)
template <bool RBN, typename T = uint16_t, bool P3 = false>
__global__ __launch_bounds__(256) void bn_apply_acc_kernel(
    const T* __restrict__ x, int ldx, void* __restrict__ yv, int ldy, const void* __restrict__ resv,
    int ldr, int M, int C, int CVB, const float* __restrict__ acc, int R, float eps, float momentum,
    const float* __restrict__ gamma, const float* __restrict__ beta, int relu, float* saved_mean,
    float* saved_invstd, float* run_mean, float* run_var, const float* shift, ResBN rb, int64_t yps, int64_t rps) {
  constexpr bool RP3 = P3 && !RBN;  // residual planes
  T* __restrict__ y = reinterpret_cast<T*>(yv);
  const T* __restrict__ res = reinterpret_cast<const T*>(resv);
  extern __shared__ __attribute__((aligned(16))) float sums[];  // [2][CB] coefficients (+ the residual BN's)
  const GroupMap gm = groupmap(CVB);
  const bool active = gm.r0 < gm.rows;
  const int cl = (threadIdx.x % CVB) * 8;
  constexpr uint32_t E = Act8<T>::ESZ;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, rsrc_bytes(M, ldx, E));
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(res != nullptr ? resv : x, rsrc_bytes(M, res != nullptr ? ldr : ldx, RP3 ? 2 : E));
  const uint16_t* r16 = reinterpret_cast<const uint16_t*>(resv);
  const __amdgpu_buffer_rsrc_t rr1 = make_rsrc(RP3 && res != nullptr ? r16 + rps : resv, rsrc_bytes(M, ldr, 2));
  const __amdgpu_buffer_rsrc_t rr2 = make_rsrc(RP3 && res != nullptr ? r16 + 2 * rps : resv, rsrc_bytes(M, ldr, 2));
  const int stride = gridDim.x * gm.rows;
  int m0 = blockIdx.x * gm.rows + gm.r0;
  Act8<T> xv[BN_U], rv[BN_U];
  u32x4 rp[RP3 ? BN_U : 1][3];
  auto load_rows = [&](int mb) {
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      int m = mb + u * stride;
      xv[u].load(xr, m < M ? (uint32_t)((size_t)m * ldx + gm.cv * 8) * E : HCB_OOB);
      if (res != nullptr) {
        if constexpr (RP3) {
          const uint32_t o = m < M ? (uint32_t)((size_t)m * ldr + gm.cv * 8) * 2u : HCB_OOB;
          rp[u][0] = buf_load16(rr, o);
          rp[u][1] = buf_load16(rr1, o);
          rp[u][2] = buf_load16(rr2, o);
        } else {
          rv[u].load(rr, m < M ? (uint32_t)((size_t)m * ldr + gm.cv * 8) * E : HCB_OOB);
        }
      }
    }
  };
  // First rows are in flight while the block derives its channel coefficients (bn_coef_fwd).
  if (active) load_rows(m0);
  const bool pub = blockIdx.x == 0;
  const int t = threadIdx.x;
  auto coef = [&](auto r8) {
    constexpr bool R8 = decltype(r8)::value;
    if (!RBN || t < 128)  // RBN: the two BNs' channels on the two halves of the block, concurrently
      bn_coef_fwd<R8>(acc, R, C, gm.c0, gm.CB, M, eps, momentum, gamma, beta, shift, pub, saved_mean, saved_invstd,
                      run_mean, run_var, sums, t, RBN ? 128 : 256);
    else
      bn_coef_fwd<R8>(rb.acc, R, C, gm.c0, gm.CB, M, eps, momentum, rb.gamma, rb.beta, rb.shift, pub, rb.saved_mean,
                      rb.saved_invstd, rb.run_mean, rb.run_var, sums + 2 * gm.CB, t - 128, 128);
  };
  if (R == 8)
    coef(std::true_type{});
  else
    coef(std::false_type{});
  __syncthreads();
  if (!active) return;
  float sc[8], sh[8], sc2[RBN ? 8 : 1], sh2[RBN ? 8 : 1];
  lds_read8(sums + cl, sc);
  lds_read8(sums + gm.CB + cl, sh);
  if constexpr (RBN) {
    lds_read8(sums + 2 * gm.CB + cl, sc2);
    lds_read8(sums + 3 * gm.CB + cl, sh2);
  }
  for (; m0 < M; m0 += BN_U * stride) {
    if (m0 != blockIdx.x * gm.rows + gm.r0) load_rows(m0);
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      int m = m0 + u * stride;
      float f[8];
      xv[u].to_f(f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = f[e] * sc[e] + sh[e];
      if (res != nullptr) {
        float r[8];
        if constexpr (RP3)
          merge_p3(rp[u][0], rp[u][1], rp[u][2], r);
        else
          rv[u].to_f(r);
        if constexpr (RBN) {
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += r[e] * sc2[e] + sh2[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += r[e];
        }
      }
      if (relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
      }
      if (m < M) {
        if constexpr (P3)
          store_p3(reinterpret_cast<uint16_t*>(yv) + (size_t)m * ldy + gm.cv * 8, yps, f);
        else
          Act8<T>::store(y + (size_t)m * ldy + gm.cv * 8, f);
      }
    }
  }
}

template <typename T = uint16_t, typename TY = T, bool POOL = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce_acc_kernel(
    const T* __restrict__ dy, int lddy, const TY* __restrict__ y, int ldyv,
    const T* __restrict__ x, int ldx, int M, int C, int CVB, const float* mean, const float* invstd,
    const float* gamma, const float* beta, int relu, float* acc, int R, T* gout, int ldg, PoolSrc pool) {
  constexpr uint32_t E = Act8<T>::ESZ;
  extern __shared__ __attribute__((aligned(16))) float lds_f[];  // [2][rows][CB] partials, [4][CB] coefficients
  const GroupMap gm = groupmap(CVB);
  const bool active = gm.r0 < gm.rows;
  float s1[8] = {0}, s2[8] = {0};
  float* coef = lds_f + 2 * gm.rows * gm.CB;  // mean invstd scale shift, one thread per channel
  for (int i = threadIdx.x; i < gm.CB; i += blockDim.x) {
    const int c = gm.c0 + i;
    const float mu = mean[c], is = invstd[c];
    const float sc = gamma[c] * is;
    coef[i] = mu;
    coef[gm.CB + i] = is;
    coef[2 * gm.CB + i] = sc;
    coef[3 * gm.CB + i] = beta[c] - mu * sc;
  }
  __syncthreads();
  if (active) {
    const int cl = (threadIdx.x % CVB) * 8;
    float mu[8], is[8], sc[8], sh[8];
    lds_read8(coef + cl, mu);
    lds_read8(coef + gm.CB + cl, is);
    lds_read8(coef + 2 * gm.CB + cl, sc);
    lds_read8(coef + 3 * gm.CB + cl, sh);
    constexpr uint32_t EY = Act8<TY>::ESZ;
    BwdSrcT<T, TY, POOL> src{make_rsrc(POOL ? x : dy, rsrc_bytes(M, POOL ? ldx : lddy, E)),
                             make_rsrc(x, rsrc_bytes(M, ldx, E)),
                             y != nullptr ? make_rsrc(y, rsrc_bytes(M, ldyv, EY)) : make_rsrc(x, rsrc_bytes(M, ldx, E)),
                             lddy, ldx, ldyv, gm.cv, pool};
    const int stride = gridDim.x * gm.rows;
    for (int m0 = blockIdx.x * gm.rows + gm.r0; m0 < M; m0 += BN_UB * stride) {
      Act8<T> dv[BN_UB], xv[BN_UB];
      Act8<TY> yv[BN_UB];
#pragma unroll
      for (int u = 0; u < BN_UB; ++u) src.load(m0 + u * stride, M, relu, dv[u], xv[u], yv[u]);
#pragma unroll
      for (int u = 0; u < BN_UB; ++u) {
        const int m = m0 + u * stride;
        float g[8], xh[8];
        bwd_math_t<T, TY>(dv[u], xv[u], yv[u], relu, mu, is, sc, sh, g, xh);
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // rows beyond M load zeros: g = 0 contributes nothing
          s1[e] += g[e];
          s2[e] += g[e] * xh[e];
        }
        if (gout != nullptr && m < M) Act8<T>::store(gout + (size_t)m * ldg + gm.cv * 8, g);
      }
    }
  }
  // block partial -> LDS rows -> column sums -> atomics into replica blockIdx.x % R
  const int cl = (threadIdx.x % CVB) * 8;
  if (active) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lds_f[gm.r0 * gm.CB + cl + e] = s1[e];
      lds_f[gm.rows * gm.CB + gm.r0 * gm.CB + cl + e] = s2[e];
    }
  }
  __syncthreads();
  float* dst = acc + (size_t)(blockIdx.x % R) * 2 * C;
  for (int i = threadIdx.x; i < gm.CB; i += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < gm.rows; ++r) {
      a += lds_f[r * gm.CB + i];
      b += lds_f[gm.rows * gm.CB + r * gm.CB + i];
    }
    atomicAdd(dst + gm.c0 + i, a);
    atomicAdd(dst + C + gm.c0 + i, b);
  }
}

// backward coefficients of the block's channel group: [6][CB] mean invstd scale shift k1 k2 (k1, k2:
// the dbeta / dgamma sums over M); block 0 publishes dgamma / dbeta and the next step's shift
template <bool R8>
__device__ __forceinline__ void bn_coef_bwd(const float* __restrict__ acc, int R, int C, int c0, int CB, int M,
                                            const float* mean, const float* invstd, const float* gamma,
                                            const float* beta, float* dgamma, float* dbeta, float* shift_out,
                                            float* coef) {
  const float invM = 1.f / (float)M;
  for (int i = threadIdx.x; i < CB; i += blockDim.x) {
    const int c = c0 + i;
    float sb, sg;
    sum_replicas2<R8>(acc, R, C, c, sb, sg);
    const float mu = mean[c], is = invstd[c];
    const float sc = gamma[c] * is;
    coef[i] = mu;
    coef[CB + i] = is;
    coef[2 * CB + i] = sc;
    coef[3 * CB + i] = beta[c] - mu * sc;
    coef[4 * CB + i] = sb * invM;
    coef[5 * CB + i] = sg * invM;
    if (blockIdx.x == 0) {
      dbeta[c] = sb;
      dgamma[c] = sg;
      // this step's batch mean becomes the next step's statistic shift (the forward readers of
      // the shift have all run: no block of this launch reads it)
      if (shift_out != nullptr) shift_out[c] = mu;
    }
  }
}

// P3 (fp32 path): dx is written as bf16 hi / mid / lo planes (plane stride dxps elements), the
// operand format of the data- and weight-gradient GEMMs that consume it
// ADD: dx = BN-backward(dy) + addend (row stride ldadd, T) -- a pre-activation BN on an identity
// shortcut (ResNet v2: d(block input) = BN'(d preact) + d(block output)) in the same pass
template <typename T = uint16_t, typename TY = T, bool P3 = false, bool POOL = false, bool ADD = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_acc_kernel(
    const T* __restrict__ dy, int lddy, const TY* __restrict__ y, int ldyv,
    const T* __restrict__ x, int ldx, void* __restrict__ dxv, int lddx, int M, int C, int CVB,
    const float* mean, const float* invstd, const float* gamma, const float* beta, const float* __restrict__ acc,
    int R, float* dgamma, float* dbeta, int relu, float* shift_out, int64_t dxps, PoolSrc pool,
    const T* __restrict__ addp, int ldadd) {
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [6][CB]: mean invstd scale shift k1 k2
  const GroupMap gm = groupmap(CVB);
  const bool active = gm.r0 < gm.rows;
  constexpr uint32_t E = Act8<T>::ESZ, EY = Act8<TY>::ESZ;
  T* __restrict__ dx = reinterpret_cast<T*>(dxv);
  BwdSrcT<T, TY, POOL> src{make_rsrc(POOL ? x : dy, rsrc_bytes(M, POOL ? ldx : lddy, E)),
                           make_rsrc(x, rsrc_bytes(M, ldx, E)),
                           y != nullptr ? make_rsrc(y, rsrc_bytes(M, ldyv, EY)) : make_rsrc(x, rsrc_bytes(M, ldx, E)),
                           lddy, ldx, ldyv, gm.cv, pool};
  const int stride = gridDim.x * gm.rows;
  const int mfirst = blockIdx.x * gm.rows + gm.r0;
  Act8<T> dv[BN_UB], xv[BN_UB];
  Act8<TY> yv[BN_UB];
  // First rows are in flight while the block derives its channel coefficients: thread i < CB
  // reduces channel c0 + i's dbeta / dgamma replicas and folds its parameters into LDS
  if (active) {
#pragma unroll
    for (int u = 0; u < BN_UB; ++u) src.load(mfirst + u * stride, M, relu, dv[u], xv[u], yv[u]);
  }
  if (R == 8)
    bn_coef_bwd<true>(acc, R, C, gm.c0, gm.CB, M, mean, invstd, gamma, beta, dgamma, dbeta, shift_out, coef);
  else
    bn_coef_bwd<false>(acc, R, C, gm.c0, gm.CB, M, mean, invstd, gamma, beta, dgamma, dbeta, shift_out, coef);
  __syncthreads();
  if (!active) return;
  const int cl = (threadIdx.x % CVB) * 8;
  float mu[8], is[8], sc[8], sh[8], k1[8], k2[8];
  lds_read8(coef + cl, mu);
  lds_read8(coef + gm.CB + cl, is);
  lds_read8(coef + 2 * gm.CB + cl, sc);
  lds_read8(coef + 3 * gm.CB + cl, sh);
  lds_read8(coef + 4 * gm.CB + cl, k1);
  lds_read8(coef + 5 * gm.CB + cl, k2);
  const __amdgpu_buffer_rsrc_t adr = make_rsrc(ADD ? (const void*)addp : (const void*)x,
                                               rsrc_bytes(M, ADD ? ldadd : ldx, E));
  for (int m0 = mfirst; m0 < M; m0 += BN_UB * stride) {
    if (m0 != mfirst) {
#pragma unroll
      for (int u = 0; u < BN_UB; ++u) src.load(m0 + u * stride, M, relu, dv[u], xv[u], yv[u]);
    }
    Act8<T> av[ADD ? BN_UB : 1];
    if constexpr (ADD) {
#pragma unroll
      for (int u = 0; u < BN_UB; ++u) {
        const int m = m0 + u * stride;
        av[u].load(adr, m < M ? (uint32_t)((size_t)m * ldadd + gm.cv * 8) * E : HCB_OOB);
      }
    }
#pragma unroll
    for (int u = 0; u < BN_UB; ++u) {
      const int m = m0 + u * stride;
      float g[8], xh[8], o[8];
      bwd_math_t<T, TY>(dv[u], xv[u], yv[u], relu, mu, is, sc, sh, g, xh);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = sc[e] * (g[e] - k1[e] - xh[e] * k2[e]);
      if constexpr (ADD) {
        float a[8];
        av[u].to_f(a);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += a[e];
      }
      if (m < M) {
        if constexpr (P3)
          store_p3(reinterpret_cast<uint16_t*>(dxv) + (size_t)m * lddx + gm.cv * 8, dxps, o);
        else
          Act8<T>::store(dx + (size_t)m * lddx + gm.cv * 8, o);
      }
    }
  }
}

// ResNet stem: BN (statistics from the conv epilogue's replicas) + ReLU + max pool in one pass.
// The BN+ReLU output is never written: each thread normalises the (<= kh x kw) window elements
// of one pooled pixel x 8 channels, keeps the max and the first-max window position (the
// argmax the pool backward gathers with), and stores only the pooled tensor. The backward
// recomputes the ReLU mask from z (mode 2), so nothing else needs the full-size activation.
// K3: the 3x3 window unrolled, its 9 loads in flight together (buffer loads, out-of-image taps
// excluded by a select) instead of one dependent loop trip per tap.
// P3 (fp32 path): the pooled output is written as bf16 hi / mid / lo planes (plane stride yps)
template <bool K3, typename T = uint16_t, bool P3 = false>
__global__ __launch_bounds__(256) void bn_relu_maxpool_acc_kernel(
    const T* __restrict__ z, int H, int W, int C, int CVB, void* __restrict__ yv, int P, int Q, int ldy,
    uint8_t* __restrict__ amax, int kh, int kw, int sh, int sw, int ph, int pw, int Nimg, int M,
    const float* __restrict__ acc, int R, float eps, float momentum, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* saved_mean, float* saved_invstd, float* run_mean, float* run_var,
    const float* shift, int64_t yps) {
  T* __restrict__ y = reinterpret_cast<T*>(yv);
  extern __shared__ __attribute__((aligned(16))) float sums[];  // [2][CB]
  const GroupMap gm = groupmap(CVB);
  // channel coefficients once per block channel, one round trip, in LDS (bn_coef_fwd)
  if (R == 8)
    bn_coef_fwd<true>(acc, R, C, gm.c0, gm.CB, M, eps, momentum, gamma, beta, shift, blockIdx.x == 0, saved_mean,
                      saved_invstd, run_mean, run_var, sums, threadIdx.x, 256);
  else
    bn_coef_fwd<false>(acc, R, C, gm.c0, gm.CB, M, eps, momentum, gamma, beta, shift, blockIdx.x == 0, saved_mean,
                       saved_invstd, run_mean, run_var, sums, threadIdx.x, 256);
  __syncthreads();
  if (gm.r0 >= gm.rows) return;
  float sc[8], sft[8];
  const int cl = (threadIdx.x % CVB) * 8;
  lds_read8(sums + cl, sc);
  lds_read8(sums + gm.CB + cl, sft);
  const unsigned PQ = (unsigned)P * Q, total = (unsigned)Nimg * PQ;
  for (unsigned op = blockIdx.x * gm.rows + gm.r0; op < total; op += gridDim.x * gm.rows) {
    const int n = (int)(op / PQ);
    const int rem = (int)(op - (unsigned)n * PQ);
    const int p = rem / Q, q = rem - p * Q;
    const int h0 = p * sh - ph, w0 = q * sw - pw;
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      arg[e] = 255;
    }
    if constexpr (K3) {
      constexpr uint32_t E = Act8<T>::ESZ;
      const __amdgpu_buffer_rsrc_t zr = make_rsrc(z, (uint32_t)M * (uint32_t)C * E);
      const int base = ((n * H + h0) * W + w0) * C + gm.cv * 8;  // element offset of tap (0, 0)
      Act8<T> v[9];
      bool okt[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          okt[r * 3 + t] = (unsigned)(h0 + r) < (unsigned)H && (unsigned)(w0 + t) < (unsigned)W;
          v[r * 3 + t].load(zr, okt[r * 3 + t] ? (uint32_t)(base + (r * W + t) * C) * E : HCB_OOB);
        }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        float f[8];
        v[k].to_f(f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float val = okt[k] ? fmaxf(f[e] * sc[e] + sft[e], 0.f) : -INFINITY;
          if (val > best[e]) {  // strict: the FIRST maximal element keeps the gradient
            best[e] = val;
            arg[e] = k;
          }
        }
      }
    } else
    for (int r = 0; r < kh; ++r) {
      const int h = h0 + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < kw; ++s) {
        const int w = w0 + s;
        if ((unsigned)w >= (unsigned)W) continue;
        float f[8];
        Act8<T> zv;
        zv.load(z + ((size_t)(n * H + h) * W + w) * C + gm.cv * 8);
        zv.to_f(f);
        const int pos = r * kw + s;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = fmaxf(f[e] * sc[e] + sft[e], 0.f);
          if (v > best[e]) {  // strict: the FIRST maximal element keeps the gradient
            best[e] = v;
            arg[e] = pos;
          }
        }
      }
    }
    if constexpr (P3)
      store_p3(reinterpret_cast<uint16_t*>(yv) + (size_t)op * ldy + gm.cv * 8, yps, best);
    else
      Act8<T>::store(y + (size_t)op * ldy + gm.cv * 8, best);
    u32x2 a;
    a[0] = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a[1] = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *reinterpret_cast<u32x2*>(amax + (size_t)op * C + gm.cv * 8) = a;
  }
}

// (row splits) x (channel groups); ~2048 blocks in total, each thread >= 1 row
static dim3 bn_grid_groups(int M, int C, int* cvb_out) {
  const int CV = C / 8;
  const int cvb = bn_group_vecs(CV);
  const int groups = CV / cvb;
  const int rows = 256 / cvb;
  int need = (M + rows - 1) / rows;
  static const int blocks = [] {
    const char* e = getenv("HCB_BN_BLOCKS");
    return e != nullptr && atoi(e) > 0 ? atoi(e) : 2048;
  }();
  int target = blocks / groups;
  if (target < 1) target = 1;
  // Small tensors: give every thread up to BN_U rows (all loads in flight at once) rather than
  // one row per thread -- fewer workgroups to dispatch and one memory round trip, while the
  // grid still covers every CU.
  static const int rpt = [] {
    const char* e = getenv("HCB_BN_RPT");
    return e != nullptr && atoi(e) > 0 ? atoi(e) : BN_U;
  }();
  int floor_s = (256 + groups - 1) / groups;
  int want = (need + rpt - 1) / rpt;
  if (want < floor_s) want = floor_s < need ? floor_s : need;
  int s = want < target ? want : target;
  if (s < 1) s = 1;
  *cvb_out = cvb;
  return dim3(s, groups);
}

template <typename T, bool P3 = false>
static void bn_apply_acc_t(const void* x, int ldx, void* y, int ldy, const void* res, int ldr, int M, int C,
                           const float* acc, int R, float eps, float momentum, const float* gamma, const float* beta,
                           int relu, float* saved_mean, float* saved_invstd, float* run_mean, float* run_var,
                           const float* shift, const ResBN* res_bn, hipStream_t st, int64_t yps, int64_t rps) {
  int cvb;
  dim3 grid = bn_grid_groups(M, C, &cvb);
  const ResBN rb = res_bn != nullptr ? *res_bn : ResBN{};
  if (res_bn != nullptr)
    hipLaunchKernelGGL((bn_apply_acc_kernel<true, T, P3>), grid, dim3(256), (size_t)4 * cvb * 8 * 4, st, (const T*)x,
                       ldx, y, ldy, res, ldr, M, C, cvb, acc, R, eps, momentum, gamma, beta, relu, saved_mean,
                       saved_invstd, run_mean, run_var, shift, rb, yps, rps);
  else
    hipLaunchKernelGGL((bn_apply_acc_kernel<false, T, P3>), grid, dim3(256), (size_t)2 * cvb * 8 * 4, st, (const T*)x,
                       ldx, y, ldy, res, ldr, M, C, cvb, acc, R, eps, momentum, gamma, beta, relu, saved_mean,
                       saved_invstd, run_mean, run_var, shift, rb, yps, rps);
}
void launch_bn_apply_acc(const void* x, int ldx, void* y, int ldy, const void* res, int ldr, int M, int C,
                         const float* acc, int R, float eps, float momentum, const float* gamma, const float* beta,
                         int relu, float* saved_mean, float* saved_invstd, float* run_mean, float* run_var,
                         const float* shift, const ResBN* res_bn, hipStream_t st, bool f32, int64_t yps, int64_t rps) {
  auto fn = yps > 0 ? bn_apply_acc_t<float, true> : (f32 ? bn_apply_acc_t<float> : bn_apply_acc_t<uint16_t>);
  fn(x, ldx, y, ldy, res, ldr, M, C, acc, R, eps, momentum, gamma, beta, relu, saved_mean, saved_invstd, run_mean,
     run_var, shift, res_bn, st, yps, rps);
}

void launch_bn_relu_maxpool_acc(const void* z, int N, int H, int W, int C, void* y, int P, int Q, int ldy, void* amax,
                                int kh, int kw, int sh, int sw, int ph, int pw, const float* acc, int R, float eps,
                                float momentum, const float* gamma, const float* beta, float* saved_mean,
                                float* saved_invstd, float* run_mean, float* run_var, const float* shift,
                                hipStream_t st, bool f32, int64_t yps) {
  int cvb;
  dim3 grid = bn_grid_groups(N * P * Q, C, &cvb);
  const bool k3 = kh == 3 && kw == 3 && (long)N * H * W * C * (f32 ? 2 : 1) < (1l << 30);
  if (f32 && yps > 0)
    hipLaunchKernelGGL((k3 ? bn_relu_maxpool_acc_kernel<true, float, true> : bn_relu_maxpool_acc_kernel<false, float, true>),
                       grid, dim3(256), (size_t)2 * cvb * 8 * 4, st, (const float*)z, H, W, C, cvb, y, P, Q, ldy,
                       (uint8_t*)amax, kh, kw, sh, sw, ph, pw, N, N * H * W, acc, R, eps, momentum, gamma, beta,
                       saved_mean, saved_invstd, run_mean, run_var, shift, yps);
  else if (f32)
    hipLaunchKernelGGL((k3 ? bn_relu_maxpool_acc_kernel<true, float> : bn_relu_maxpool_acc_kernel<false, float>), grid,
                       dim3(256), (size_t)2 * cvb * 8 * 4, st, (const float*)z, H, W, C, cvb, y, P, Q, ldy,
                       (uint8_t*)amax, kh, kw, sh, sw, ph, pw, N, N * H * W, acc, R, eps, momentum, gamma, beta,
                       saved_mean, saved_invstd, run_mean, run_var, shift, (int64_t)0);
  else
    hipLaunchKernelGGL(k3 ? bn_relu_maxpool_acc_kernel<true> : bn_relu_maxpool_acc_kernel<false>, grid, dim3(256),
                       (size_t)2 * cvb * 8 * 4, st, (const uint16_t*)z, H, W, C, cvb, y, P, Q, ldy,
                       (uint8_t*)amax, kh, kw, sh, sw, ph, pw, N, N * H * W, acc, R, eps, momentum, gamma, beta,
                       saved_mean, saved_invstd, run_mean, run_var, shift, (int64_t)0);
}

void launch_bn_bwd_reduce_acc(const void* dy, int lddy, const void* y, int ldyv, const void* x, int ldx, int M,
                              int C, const float* mean, const float* invstd, const float* gamma, const float* beta,
                              int relu, float* acc, int R, void* gout, int ldg, hipStream_t st, bool f32, bool yh,
                              const PoolSrc* pool) {
  int cvb;
  dim3 grid = bn_grid_groups(M, C, &cvb);
  // every block adds into replica blockIdx.x % R; deterministic mode: at most R row blocks, so
  // each replica slot gets one add (the kernel strides over the rows with any grid)
  if (deterministic() && (int)grid.x > R) grid.x = R;
  size_t lds = ((size_t)2 * (256 / cvb) + 4) * cvb * 8 * 4;
  const PoolSrc ps = pool != nullptr ? *pool : PoolSrc{};
  if (pool != nullptr && f32)
    hipLaunchKernelGGL((bn_bwd_reduce_acc_kernel<float, float, true>), grid, dim3(256), lds, st, (const float*)dy,
                       lddy, (const float*)y, ldyv, (const float*)x, ldx, M, C, cvb, mean, invstd, gamma, beta, relu,
                       acc, R, (float*)gout, ldg, ps);
  else if (pool != nullptr)
    hipLaunchKernelGGL((bn_bwd_reduce_acc_kernel<uint16_t, uint16_t, true>), grid, dim3(256), lds, st,
                       (const uint16_t*)dy, lddy, (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx, M, C, cvb, mean,
                       invstd, gamma, beta, relu, acc, R, (uint16_t*)gout, ldg, ps);
  else if (f32 && yh)
    hipLaunchKernelGGL((bn_bwd_reduce_acc_kernel<float, uint16_t>), grid, dim3(256), lds, st, (const float*)dy, lddy,
                       (const uint16_t*)y, ldyv, (const float*)x, ldx, M, C, cvb, mean, invstd, gamma, beta, relu, acc,
                       R, (float*)gout, ldg, ps);
  else if (f32)
    hipLaunchKernelGGL(bn_bwd_reduce_acc_kernel<float>, grid, dim3(256), lds, st, (const float*)dy, lddy,
                       (const float*)y, ldyv, (const float*)x, ldx, M, C, cvb, mean, invstd, gamma, beta, relu, acc, R,
                       (float*)gout, ldg, ps);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_acc_kernel<uint16_t>, grid, dim3(256), lds, st, (const uint16_t*)dy, lddy,
                       (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx, M, C, cvb, mean, invstd, gamma, beta, relu,
                       acc, R, (uint16_t*)gout, ldg, ps);
}

void launch_bn_bwd_apply_acc(const void* dy, int lddy, const void* y, int ldyv, const void* x, int ldx, void* dx,
                             int lddx, int M, int C, const float* mean, const float* invstd, const float* gamma,
                             const float* beta, const float* acc, int R, float* dgamma, float* dbeta, int relu,
                             float* shift_out, hipStream_t st, bool f32, bool yh, int64_t dxps, const PoolSrc* pool,
                             const void* add, int ldadd) {
  int cvb;
  dim3 grid = bn_grid_groups(M, C, &cvb);
  const size_t lds = (size_t)6 * cvb * 8 * 4;
  const PoolSrc ps = pool != nullptr ? *pool : PoolSrc{};
  if (add != nullptr) {  // addend: plain (non-plane) dx, no pooled dy (checked on the host)
    if (f32)
      hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<float, float, false, false, true>), grid, dim3(256), lds, st,
                         (const float*)dy, lddy, (const float*)y, ldyv, (const float*)x, ldx, dx, lddx, M, C, cvb,
                         mean, invstd, gamma, beta, acc, R, dgamma, dbeta, relu, shift_out, (int64_t)0, ps,
                         (const float*)add, ldadd);
    else
      hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<uint16_t, uint16_t, false, false, true>), grid, dim3(256), lds, st,
                         (const uint16_t*)dy, lddy, (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx, dx, lddx, M, C,
                         cvb, mean, invstd, gamma, beta, acc, R, dgamma, dbeta, relu, shift_out, (int64_t)0, ps,
                         (const uint16_t*)add, ldadd);
  } else if (pool != nullptr && f32 && dxps > 0) {
    hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<float, float, true, true>), grid, dim3(256), lds, st,
                       (const float*)dy, lddy, (const float*)y, ldyv, (const float*)x, ldx, dx, lddx, M, C, cvb, mean,
                       invstd, gamma, beta, acc, R, dgamma, dbeta, relu, shift_out, dxps, ps, (const float*)nullptr, 0);
  } else if (pool != nullptr && !f32) {
    hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<uint16_t, uint16_t, false, true>), grid, dim3(256), lds, st,
                       (const uint16_t*)dy, lddy, (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx, dx, lddx, M, C,
                       cvb, mean, invstd, gamma, beta, acc, R, dgamma, dbeta, relu, shift_out, (int64_t)0, ps,
                       (const uint16_t*)nullptr, 0);
  } else if (f32 && dxps > 0) {
    if (yh)
      hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<float, uint16_t, true>), grid, dim3(256), lds, st, (const float*)dy,
                         lddy, (const uint16_t*)y, ldyv, (const float*)x, ldx, dx, lddx, M, C, cvb, mean, invstd,
                         gamma, beta, acc, R, dgamma, dbeta, relu, shift_out, dxps, ps, (const float*)nullptr, 0);
    else
      hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<float, float, true>), grid, dim3(256), lds, st, (const float*)dy,
                         lddy, (const float*)y, ldyv, (const float*)x, ldx, dx, lddx, M, C, cvb, mean, invstd, gamma,
                         beta, acc, R, dgamma, dbeta, relu, shift_out, dxps, ps, (const float*)nullptr, 0);
  } else if (f32) {
    hipLaunchKernelGGL(bn_bwd_apply_acc_kernel<float>, grid, dim3(256), lds, st, (const float*)dy, lddy,
                       (const float*)y, ldyv, (const float*)x, ldx, dx, lddx, M, C, cvb, mean, invstd, gamma, beta, acc,
                       R, dgamma, dbeta, relu, shift_out, (int64_t)0, ps, (const float*)nullptr, 0);
  } else {
    hipLaunchKernelGGL(bn_bwd_apply_acc_kernel<uint16_t>, grid, dim3(256), lds, st, (const uint16_t*)dy, lddy,
                       (const uint16_t*)y, ldyv, (const uint16_t*)x, ldx, dx, lddx, M, C, cvb, mean, invstd, gamma,
                       beta, acc, R, dgamma, dbeta, relu, shift_out, (int64_t)0, ps, (const uint16_t*)nullptr, 0);
  }
}

// Standalone BN statistics into the R accumulator replicas, for a BN whose input has no producing
// GEMM epilogue to fuse them into (ResNet v2's pre-activation and final BN: the input is a block
// output, conv + shortcut): sums of (v - K) and (v - K)^2 per channel, K = the layer's previous batch
// mean (shift; 0 when null), block partials through LDS, then atomics into replica blockIdx.x % R --
// exactly what a conv epilogue leaves for bn_apply_acc.
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_acc_kernel(const T* __restrict__ x, int ldx, int M, int C, int CVB,
                                                           const float* __restrict__ shift, float* acc, int R) {
  constexpr uint32_t E = Act8<T>::ESZ;
  extern __shared__ __attribute__((aligned(16))) float lds_f[];  // [2][rows][CB]
  const GroupMap gm = groupmap(CVB);
  const bool active = gm.r0 < gm.rows;
  const int cl = (threadIdx.x % CVB) * 8;
  float s1[8] = {0}, s2[8] = {0};
  if (active) {
    float k[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) k[e] = shift != nullptr ? shift[gm.cv * 8 + e] : 0.f;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, rsrc_bytes(M, ldx, E));
    const int stride = gridDim.x * gm.rows;
    for (int m0 = blockIdx.x * gm.rows + gm.r0; m0 < M; m0 += BN_U * stride) {
      Act8<T> v[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const int m = m0 + u * stride;
        v[u].load(xr, m < M ? (uint32_t)((size_t)m * ldx + gm.cv * 8) * E : HCB_OOB);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        if (m0 + u * stride >= M) continue;  // an out-of-range zero row would add (-K)^2
        float f[8];
        v[u].to_f(f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = f[e] - k[e];
          s1[e] += d;
          s2[e] += d * d;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lds_f[gm.r0 * gm.CB + cl + e] = s1[e];
      lds_f[gm.rows * gm.CB + gm.r0 * gm.CB + cl + e] = s2[e];
    }
  }
  __syncthreads();
  float* dst = acc + (size_t)(blockIdx.x % R) * 2 * C;
  for (int i = threadIdx.x; i < gm.CB; i += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < gm.rows; ++r) {
      a += lds_f[r * gm.CB + i];
      b += lds_f[gm.rows * gm.CB + r * gm.CB + i];
    }
    atomicAdd(dst + gm.c0 + i, a);
    atomicAdd(dst + C + gm.c0 + i, b);
  }
}

void launch_bn_stats_acc(const void* x, int ldx, int M, int C, const float* shift, float* acc, int R, hipStream_t st,
                         bool f32) {
  int cvb;
  dim3 grid = bn_grid_groups(M, C, &cvb);
  // deterministic mode: at most R row blocks, so each replica slot receives a single add
  if (deterministic() && (int)grid.x > R) grid.x = R;
  const size_t lds = (size_t)2 * (256 / cvb) * cvb * 8 * 4;
  if (f32)
    hipLaunchKernelGGL(bn_stats_acc_kernel<float>, grid, dim3(256), lds, st, (const float*)x, ldx, M, C, cvb, shift,
                       acc, R);
  else
    hipLaunchKernelGGL(bn_stats_acc_kernel<uint16_t>, grid, dim3(256), lds, st, (const uint16_t*)x, ldx, M, C, cvb,
                       shift, acc, R);
}

}  // namespace hcb
