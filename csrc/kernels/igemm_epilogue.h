// Shared epilogue of the implicit-GEMM conv kernels: fp32 accumulators -> (fused BN
// statistics from registers) -> LDS staging (padded fp32 rows) -> coalesced 16-byte stores
// with optional beta-accumulate, bias, fp32 output and strided-output pixel remap.
#pragma once
#include "common.h"
#include "kernels.h"

namespace hcb {

// Bytes of LDS the epilogue needs for a BM x BN tile computed by WM x WN waves.
constexpr size_t igemm_epilogue_lds(int BM, int BN, int WM) {
  return (size_t)BM * (BN + 4) * 4 + (size_t)WM * 2 * BN * 4;
}

template <int WM, int WN, int TM, int TN>
__device__ __forceinline__ void igemm_epilogue(const ConvParams& p, f32x4 (&acc)[TM / 16][TN / 16], char* smem,
                                               int tm, int m0, int n0, int wm, int wn, int lane, int tid) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int LDC = BN + 4;
  const int frow = lane & 15, fq = lane >> 4;
  float* Cs = reinterpret_cast<float*>(smem);
  float* red = Cs + BM * LDC;  // [WM][2][BN] per-wave column partial sums
  if (p.stats != nullptr) {
    // per-column partial BN statistics straight from the accumulators (rows beyond M are
    // exact zeros): sum the wave's row quads in registers, then across the 4 lane groups
    // that share a column with two xor-shuffles.
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[i][j][e];
          s1 += v;
          s2 += v * v;
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
  __syncthreads();

  if (p.stats != nullptr) {
    for (int col = tid; col < BN; col += 256) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s1 += red[(w * 2) * BN + col];
        s2 += red[(w * 2 + 1) * BN + col];
      }
      int gc = n0 + col;
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

  const int PQ = p.P * p.Q;
  constexpr int SEGS = BN / 8;
  for (int sidx = tid; sidx < BM * SEGS; sidx += 256) {
    int row = sidx / SEGS, cs = sidx - row * SEGS;
    int m = m0 + row;
    int col = n0 + cs * 8;
    if (m >= p.M || col >= p.Nout) continue;
    size_t orow = (size_t)m;
    if (p.remap) {
      int n = m / PQ, r = m - n * PQ;
      int pp = r / p.Q, qq = r - pp * p.Q;
      orow = ((size_t)n * p.OH + (size_t)pp * p.osh) * p.OW + (size_t)qq * p.osw;
    }
    float v[8];
    const f32x4* src = reinterpret_cast<const f32x4*>(Cs + row * LDC + cs * 8);
    f32x4 v0 = src[0], v1 = src[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = v0[e];
      v[4 + e] = v1[e];
    }
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
    } else {
      uint16_t* yo = reinterpret_cast<uint16_t*>(p.y) + orow * p.ldy + col;
      if (p.beta) {
        const uint16_t* yi = reinterpret_cast<const uint16_t*>(p.yres) + orow * p.ldy + col;
        float o[8];
        unpack8(*reinterpret_cast<const u32x4*>(yi), o);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += o[e];
      }
      *reinterpret_cast<u32x4*>(yo) = pack8(v);
    }
  }
}

}  // namespace hcb
