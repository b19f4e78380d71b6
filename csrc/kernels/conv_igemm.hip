// Implicit-GEMM convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16.
//
//   C[M = N*P*Q, Nout] = im2col(X)[M, K = R*S*Cin] * W[Nout, K]^T
//
// One kernel family serves three roles of the reference's MKL-DNN primitives
// ("Conv2D fwd / bwd-data", driven by tf_cnn_benchmarks at
// /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81):
//   * forward conv                     (X = activations, W = KRSC weights)
//   * data-gradient conv               (X = dY, W = flipped/transposed weights, optional
//                                       lhs-dilation for strided convs, or an output
//                                       pixel remap for strided 1x1 convs)
//   * the FC layer                     (H = W = 1, fp32 output + bias)
//
// Design (MI355X-first, not a translation):
//   * 256 threads = 4 waves of 64, wave tile TMxTN built from 16x16x32 bf16 MFMAs
//     (fp32 accumulate), block tile BM x BN x BK=64.
//   * im2col is never materialised: each thread gathers 16-byte channel vectors of
//     the input with raw buffer loads; halo / padding / tail rows use an out-of-range
//     offset, which the buffer unit turns into zeros (no branches around loads).
//   * register-staged double-buffered LDS (issue the next tile's global loads before
//     the MFMAs, write them to the other LDS buffer after), one barrier per k-step.
//   * LDS rows are 128 B (BK=64 bf16); 16-byte chunks are XOR-swizzled with
//     (row>>1)&7 so the ds_read_b128 fragment reads are bank-conflict free.
//   * XCD-aware block remap so neighbouring tiles (sharing the im2col panel) sit on
//     one XCD's L2.
//   * epilogue staged through LDS as fp32: fully coalesced 16-byte bf16 stores,
//     optional beta-accumulate, bias, fp32 output and fused per-channel BatchNorm
//     statistics (sum / sum of squares per M-tile, reduced later in fp64).
#include "common.h"
#include "kernels.h"

namespace hcb {

template <int WM, int WN, int TM, int TN, bool CBIG, bool LHSDIL>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN, BK = 64;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AV = BM / 32, BV = BN / 32;  // 16-byte vectors per thread per k-step
  static_assert(WM * WN == 4, "4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u32x4* As = reinterpret_cast<u32x4*>(smem);  // [2][BM*8]
  u32x4* Bs = As + 2 * BM * 8;                 // [2][BN*8]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int chunk = tid & 7;

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, p.w_bytes);

  // ---- per-thread A row decode (fixed for the whole K loop)
  int a_pix[AV], a_h0[AV], a_w0[AV];
  const int PQ = p.P * p.Q;
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    int m = m0 + (tid >> 3) + 32 * v;
    if (m < p.M) {
      int n = m / PQ, r = m - n * PQ;
      int pp = r / p.Q, qq = r - pp * p.Q;
      a_pix[v] = n * p.H * p.W;
      a_h0[v] = pp * p.stride_h - p.pad_h;
      a_w0[v] = qq * p.stride_w - p.pad_w;
    } else {
      a_pix[v] = -1;
      a_h0[v] = 0;
      a_w0[v] = 0;
    }
  }
  uint32_t b_off[BV];
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    int j = n0 + (tid >> 3) + 32 * v;
    b_off[v] = (j < p.Nout) ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
  }

  u32x4 ra[AV], rb[BV];
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int RS = p.R * p.S;
  auto gload = [&](int kt) {
    const int k0 = kt * BK;
    int tap, c;
    if constexpr (CBIG) {
      tap = k0 / p.C;
      c = k0 - tap * p.C + chunk * 8;
    } else {
      int k = k0 + chunk * 8;
      tap = k / p.C;
      c = k - tap * p.C;
    }
    const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
    const bool tap_ok = tap < RS;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      int h = a_h0[v] + r * p.dil_h;
      int w = a_w0[v] + s * p.dil_w;
      bool ok = tap_ok && a_pix[v] >= 0 && h >= 0 && w >= 0;
      if constexpr (LHSDIL) {
        ok = ok && (h % p.idil_h == 0) && (w % p.idil_w == 0);
        h /= p.idil_h;
        w /= p.idil_w;
      }
      ok = ok && h < p.H && w < p.W;
      uint32_t off = ok ? (uint32_t)((a_pix[v] + h * p.W + w) * p.ldx + c) * 2u : HCB_OOB;
      ra[v] = buf_load16(xr, off);
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      uint32_t off = b_off[v] == HCB_OOB ? HCB_OOB : b_off[v] + (uint32_t)k0 * 2u;
      rb[v] = buf_load16(wr, off);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      int row = (tid >> 3) + 32 * v;
      As[buf * BM * 8 + row * 8 + (chunk ^ ((row >> 1) & 7))] = ra[v];
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      int row = (tid >> 3) + 32 * v;
      Bs[buf * BN * 8 + row * 8 + (chunk ^ ((row >> 1) & 7))] = rb[v];
    }
  };

  const int nk = p.Kpad / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  const int frow = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const u32x4* Ab = As + cur * BM * 8;
    const u32x4* Bb = Bs + cur * BN * 8;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int row = wm * TM + i * 16 + frow;
        int ch = ks * 4 + fq;
        u32x4 t = Ab[row * 8 + (ch ^ ((row >> 1) & 7))];
        af[i] = __builtin_bit_cast(bf16x8, t);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int row = wn * TN + j * 16 + frow;
        int ch = ks * 4 + fq;
        u32x4 t = Bb[row * 8 + (ch ^ ((row >> 1) & 7))];
        bfr[j] = __builtin_bit_cast(bf16x8, t);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS (fp32, padded rows) -> coalesced stores
  constexpr int LDC = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
  float* red = Cs + BM * LDC;  // [WM][2][BN] per-wave column partial sums
  if (p.stats != nullptr) {
    // per-column partial BN statistics straight from the accumulators (rows beyond M are
    // exact zeros): sum the wave's 4 row-quads in registers, then across the 4 lane groups
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
        p.stats[(size_t)tm * 2 * p.Nout + gc] = s1;
        p.stats[(size_t)tm * 2 * p.Nout + p.Nout + gc] = s2;
      }
    }
  }

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

template <int WM, int WN, int TM, int TN>
static void launch_cfg(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  int tiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN);
  size_t lds_main = (size_t)2 * (BM + BN) * 8 * 16;
  size_t lds_epi = (size_t)BM * (BN + 4) * 4 + (size_t)WM * 2 * BN * 4;
  size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  bool cbig = (p.C % 64) == 0;
  bool lhs = p.idil_h > 1 || p.idil_w > 1;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<WM, WN, TM, TN, true, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<WM, WN, TM, TN, true, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<WM, WN, TM, TN, false, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<WM, WN, TM, TN, false, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  if (cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, true, false>), dim3(tiles), dim3(256), lds, st, p);
  else if (cbig && lhs)
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, true, true>), dim3(tiles), dim3(256), lds, st, p);
  else if (!cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, false, false>), dim3(tiles), dim3(256), lds, st, p);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, false, true>), dim3(tiles), dim3(256), lds, st, p);
}

int conv_tile_m(int cfg) {
  switch (cfg) {
    case 0: return 128;
    case 1: return 128;
    case 2: return 64;
    case 3: return 64;
    default: return 128;
  }
}
int conv_tile_n(int cfg) {
  switch (cfg) {
    case 0: return 128;
    case 1: return 64;
    case 2: return 64;
    case 3: return 128;
    default: return 128;
  }
}

void launch_conv_igemm(const ConvParams& p, int cfg, hipStream_t st) {
  switch (cfg) {
    case 0: launch_cfg<2, 2, 64, 64>(p, st); break;   // 128 x 128
    case 1: launch_cfg<4, 1, 32, 64>(p, st); break;   // 128 x 64
    case 2: launch_cfg<2, 2, 32, 32>(p, st); break;   // 64 x 64
    case 3: launch_cfg<1, 4, 64, 32>(p, st); break;   // 64 x 128
    default: launch_cfg<2, 2, 64, 64>(p, st); break;
  }
}

}  // namespace hcb
