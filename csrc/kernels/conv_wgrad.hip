// Weight-gradient implicit GEMM on gfx950 MFMA (the MKL-DNN "Conv2D bwd-filter" role,
// SURVEY.md §2.6):
//
//   dW[i = cout][j = (r,s,c)] += sum_{m = (n,p,q)} dY[m][i] * X[n, p*sh-ph+r*dh, q*sw-pw+s*dw, c]
//
// Both operands have the reduction index (pixels) as their OUTER dimension, so they
// are staged into LDS as [64 pixels][tile cols] rows (coalesced 16-byte loads along
// channels) and the MFMA fragments are read back transposed with the gfx950 hardware
// transpose read ds_read_b64_tr_b16. LDS rows are 256 B; 32-byte slots are XOR-swizzled
// with (row&3)|((row>>1)&4) so the 8 rows touched by one 32-lane half of a transposed
// read land on 8 distinct bank groups (conflict free).
//
// The reduction (K = N*P*Q, up to 802,816 at ResNet-50 bs=64) is split across
// workgroups (split-K) so even the 64x576 stage-1 filters fill 256 CUs; partial tiles
// are staged through LDS and accumulated with fp32 atomics in 256-byte contiguous rows
// (the shape the MI355X atomic unit serves at full rate).
#include "common.h"
#include "kernels.h"

namespace hcb {

// 32-byte-slot XOR swizzle for an LDS row of NSLOT slots (NSLOT = tile cols / 16): the 8 rows
// read by one 32-lane half of a ds_read_b64_tr_b16 land on distinct bank groups.
template <int NSLOT>
__device__ __forceinline__ int wg_swz(int row) {
  if constexpr (NSLOT >= 8) return (row & 3) | ((row >> 1) & 4);
  else return ((row >> 1) & 1) | ((row >> 2) & 2);
}

template <int WM, int WN, int TM, int TN, bool CBIG>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradParams p) {
  constexpr int BM = WM * TM, BN = WN * TN, BK = 64;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AVR = BM / 8, BVR = BN / 8;        // 16-byte vectors per LDS row
  constexpr int AV = BK * AVR / 256, BV = BK * BVR / 256;  // vectors per thread
  static_assert(WM * WN == 4, "4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;                       // [2][BK][BM] bf16, 2*BM bytes per row
  char* Bs = smem + 2 * BK * BM * 2;     // [2][BK][BN]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = (p.Nout + BM - 1) / BM;
  const int tiles_n = (p.K + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int i0 = tm * BM, j0 = tn * BN;

  const int nkt = (p.M + BK - 1) / BK;
  const int kt_begin = split * p.ksteps_per_split;
  int kt_end = kt_begin + p.ksteps_per_split;
  if (kt_end > nkt) kt_end = nkt;
  if (kt_begin >= kt_end) return;  // uniform per workgroup

  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(p.dy, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);

  // A (dY) thread mapping: column vector fixed, rows vary
  const int a_cv = tid % AVR, a_r0 = tid / AVR;
  constexpr int A_RSTEP = 256 / AVR;
  const int a_col = i0 + a_cv * 8;
  const bool a_colok = a_col < p.Nout;
  // B (im2col X) thread mapping
  const int b_cv = tid % BVR, b_r0 = tid / BVR;
  constexpr int B_RSTEP = 256 / BVR;
  const int b_col = j0 + b_cv * 8;
  bool b_colok = b_col < p.K;
  int b_r = 0, b_s = 0, b_c = 0;
  if constexpr (CBIG) {
    // whole tile in one tap: computed from j0 (C % BN == 0)
    int tap = j0 / p.C;
    b_c = j0 - tap * p.C + b_cv * 8;
    b_r = tap / p.S;
    b_s = tap - b_r * p.S;
  } else {
    int tap = (int)fdiv((uint32_t)b_col, p.fd_c);
    b_c = b_col - tap * p.C;
    b_r = (int)fdiv((uint32_t)tap, p.fd_s);
    b_s = tap - b_r * p.S;
  }
  const int b_dh = b_r * p.dil_h - p.pad_h, b_dw = b_s * p.dil_w - p.pad_w;

  u32x4 ra[AV], rb[BV];
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto gload = [&](int kt) {
    const int mb = kt * BK;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      int m = mb + a_r0 + A_RSTEP * v;
      uint32_t off = (a_colok && m < p.M) ? (uint32_t)(m * p.ldy + a_col) * 2u : HCB_OOB;
      ra[v] = buf_load16(dyr, off);
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      int m = mb + b_r0 + B_RSTEP * v;
      uint32_t off = HCB_OOB;
      if (b_colok && m < p.M) {
        int n = (int)fdiv((uint32_t)m, p.fd_pq);
        int rem = m - n * p.P * p.Q;
        int pp = (int)fdiv((uint32_t)rem, p.fd_q);
        int qq = rem - pp * p.Q;
        int h = pp * p.stride_h + b_dh, w = qq * p.stride_w + b_dw;
        if (h >= 0 && h < p.H && w >= 0 && w < p.W)
          off = (uint32_t)(((n * p.H + h) * p.W + w) * p.ldx + b_c) * 2u;
      }
      rb[v] = buf_load16(xr, off);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      int row = a_r0 + A_RSTEP * v;
      int slot = (a_cv >> 1) ^ wg_swz<BM / 16>(row);
      *reinterpret_cast<u32x4*>(As + buf * BK * BM * 2 + row * BM * 2 + slot * 32 + (a_cv & 1) * 16) = ra[v];
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      int row = b_r0 + B_RSTEP * v;
      int slot = (b_cv >> 1) ^ wg_swz<BN / 16>(row);
      *reinterpret_cast<u32x4*>(Bs + buf * BK * BN * 2 + row * BN * 2 + slot * 32 + (b_cv & 1) * 16) = rb[v];
    }
  };

  const int li = lane & 15, g = lane >> 4, q4 = li >> 2, p4 = li & 3;
  // lane supplies row (row + q4), columns col + 4*p4 (col a multiple of 16); rows are NSLOT*32 B
  auto tr_read_a = [&](const char* base, int row, int col) -> short4v {
    int rr = row + q4, cb = (col + 4 * p4) * 2;
    int slot = (cb >> 5) ^ wg_swz<BM / 16>(rr);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * BM * 2 + slot * 32 + (cb & 31)));
  };
  auto tr_read_b = [&](const char* base, int row, int col) -> short4v {
    int rr = row + q4, cb = (col + 4 * p4) * 2;
    int slot = (cb >> 5) ^ wg_swz<BN / 16>(rr);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * BN * 2 + slot * 32 + (cb & 31)));
  };

  gload(kt_begin);
  lstore(0);
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int cur = (kt - kt_begin) & 1;
    if (kt + 1 < kt_end) gload(kt + 1);
    const char* Ab = As + cur * BK * BM * 2;
    const char* Bb = Bs + cur * BK * BN * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int col = wm * TM + i * 16;
        short4v lo = tr_read_a(Ab, ks * 32 + 8 * g, col);
        short4v hi = tr_read_a(Ab, ks * 32 + 8 * g + 4, col);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, t);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int col = wn * TN + j * 16;
        short4v lo = tr_read_b(Bb, ks * 32 + 8 * g, col);
        short4v hi = tr_read_b(Bb, ks * 32 + 8 * g + 4, col);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, t);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < kt_end) lstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: stage fp32 tile in LDS, then 256-byte contiguous atomic rows
  constexpr int LDC = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int row = wm * TM + i * 16 + g * 4 + e;
        int col = wn * TN + j * 16 + li;
        Cs[row * LDC + col] = acc[i][j][e];
      }
  __syncthreads();
  for (int idx = tid; idx < BM * BN; idx += 256) {
    int row = idx / BN, col = idx - row * BN;
    int gi = i0 + row, gj = j0 + col;
    if (gi < p.Nout && gj < p.K) atomicAdd(p.dw + (size_t)gi * p.K + gj, Cs[row * LDC + col]);
  }
}

template <int WM, int WN, int TM, int TN>
static void wlaunch(const WgradParams& p, int splits, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  int tiles = ((p.Nout + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  size_t lds_main = (size_t)2 * 64 * (BM + BN) * 2;
  size_t lds_epi = (size_t)BM * (BN + 4) * 4;
  size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  bool cbig = (p.C % BN) == 0;
  dim3 grid(tiles * splits);
  if (cbig) {
    static bool once = false;
    if (!once) {
      (void)hipFuncSetAttribute((const void*)conv_wgrad_kernel<WM, WN, TM, TN, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      once = true;
    }
    hipLaunchKernelGGL((conv_wgrad_kernel<WM, WN, TM, TN, true>), grid, dim3(256), lds, st, p);
  } else {
    static bool once = false;
    if (!once) {
      (void)hipFuncSetAttribute((const void*)conv_wgrad_kernel<WM, WN, TM, TN, false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      once = true;
    }
    hipLaunchKernelGGL((conv_wgrad_kernel<WM, WN, TM, TN, false>), grid, dim3(256), lds, st, p);
  }
}

int wgrad_tile_m(int cfg) { return cfg == 0 ? 128 : (cfg == 1 ? 64 : 64); }
int wgrad_tile_n(int cfg) { return cfg == 0 ? 128 : (cfg == 1 ? 128 : 64); }

void launch_conv_wgrad(const WgradParams& p, int cfg, int splits, hipStream_t st) {
  switch (cfg) {
    case 0: wlaunch<2, 2, 64, 64>(p, splits, st); break;  // 128 x 128
    case 1: wlaunch<1, 4, 64, 32>(p, splits, st); break;  // 64 x 128
    default: wlaunch<2, 2, 32, 32>(p, splits, st); break; // 64 x 64
  }
}

}  // namespace hcb
