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

#include <stdlib.h>

#include <type_traits>

namespace hcb {

// 32-byte-slot XOR swizzle for an LDS row of NSLOT slots (NSLOT = tile cols / 16): the 8 rows
// read by one 32-lane half of a ds_read_b64_tr_b16 land on distinct bank groups.
template <int NSLOT>
__device__ __forceinline__ int wg_swz(int row) {
  if constexpr (NSLOT >= 8) return (row & 3) | ((row >> 1) & 4);
  else return ((row >> 1) & 1) | ((row >> 2) & 2);
}

// Adds the LDS-staged fp32 tile into dw: a plain read-modify-write when this workgroup is the
// tile's only writer (no split-K), fp32 atomics otherwise. (Measured alternative, dropped:
// split-K partial slabs + a last-arriver sum instead of atomics was 1.2-3x slower on the
// ResNet-50 layers -- the serial tail reduction costs more than the atomics.)
__device__ __forceinline__ void wgrad_store_tile(const WgradParams& p, const float* Cs, int LDC, int BM, int BN, int i0,
                                                 int j0, int tid, int nthreads, bool sole_writer) {
  for (int idx = tid; idx < BM * BN; idx += nthreads) {
    const int row = idx / BN, col = idx - row * BN;
    const int gi = i0 + row, gj = j0 + col;
    if (gi < p.Nout && gj < p.K) {
      float* d = p.dw + (size_t)gi * p.K + gj;
      if (sole_writer)
        *d += Cs[row * LDC + col];
      else
        atomicAdd(d, Cs[row * LDC + col]);
    }
  }
}

// ---- incremental row addressing for the register-staged loaders (RI = "row-incremental").
// Both operands' rows are pixels m = (n, p, q) that advance by BK per k-step. Re-deriving
// (n, p, q) and the im2col source address of every row with magic-number divides and 32-bit
// multiplies made these k-loops VALU-bound: 40 quarter-rate integer multiplies and ~90 other
// VALU ops against 16 MFMAs per k-step in the 64x64 k-split kernel. Instead each thread keeps
// (h, w, byte offset) of its rows and adds a precomputed mixed-radix step of BK pixels
// (dn, dp, dq) with at most one carry per digit (dq < Q and dp < P): adds, two compares and
// selects. The thread -> (row, 16-byte vector) map keeps a vector's column, so its filter tap,
// fixed per thread. (The original divide-per-row loaders were measured 10-30% slower on every
// ResNet-50 layer and removed: profiles/r2p_wgrad_row_incremental.txt.)
struct WgAdvance {  // wave-uniform per-k-step increments (bytes / input rows / input cols)
  int dqw, dqo, qs, qco, dph, dpo, ps, pco, dno;
};
__device__ __forceinline__ WgAdvance wg_advance(const WgradParams& p, int rows, int esz = 2) {
  const int PQ = p.P * p.Q;
  const int dn = rows / PQ, rem = rows - dn * PQ, dp = rem / p.Q, dq = rem - dp * p.Q;
  const int pix = p.ldx * esz, rowb = p.W * pix;
  WgAdvance a;
  a.dqw = dq * p.stride_w;
  a.dqo = dq * p.stride_w * pix;
  a.qs = p.Q * p.stride_w;
  a.qco = p.stride_h * rowb - p.Q * p.stride_w * pix;  // carry into the next output row
  a.dph = dp * p.stride_h;
  a.dpo = dp * p.stride_h * rowb;
  a.ps = p.P * p.stride_h;
  a.pco = (p.H - p.P * p.stride_h) * rowb;  // carry into the next image
  a.dno = dn * p.H * rowb;
  return a;
}

template <int ROWS, int COLS, int NT>
struct WgSeg {
  static constexpr int VPR = COLS / 8;            // 16-byte vectors per LDS row
  static constexpr int V = ROWS * VPR / NT;       // vectors per thread per k-step
  // one vector of a row per thread: each load instruction then covers whole 128-byte lines
  // (VPR lanes per row) and each LDS store whole rows (conflict free). Measured: 4-vector row
  // segments per thread (a quarter of the address updates) were 10-20% SLOWER on the k-split
  // kernel -- 4x the L1 line requests per instruction and 2x LDS store conflicts.
  static constexpr int SEGV = 1;
  static constexpr int TPR = VPR / SEGV;          // threads per row
  static constexpr int RPT = V / SEGV;            // rows per thread
  static constexpr int RSTEP = NT / TPR;          // row distance between a thread's rows
  static_assert(SEGV >= 1 && SEGV <= VPR && RPT * SEGV == V && RSTEP * RPT == ROWS, "segment mapping");
  // LDS image [ROWS][COLS] bf16, 32-byte slots XOR-swizzled (wg_swz): byte offset of vector s
  // of this thread's row i (loop-invariant, hoisted by the compiler)
  __device__ __forceinline__ static int lds_off(int tid, int i, int s) {
    const int row = tid / TPR + RSTEP * i, cv = (tid % TPR) * SEGV + s;
    return row * COLS * 2 + (((cv >> 1) ^ wg_swz<COLS / 16>(row)) * 32) + (cv & 1) * 16;
  }
};

// dY operand: rows m, columns = output channels [i0, i0 + COLS). ESZ 4 (fp32 operands): a vector of 8
// values is two 16-byte loads, the second into d2
template <int ROWS, int COLS, int NT, int ESZ = 2>
struct WgALoad {
  using G = WgSeg<ROWS, COLS, NT>;
  uint32_t off[G::RPT];
  int m[G::RPT];
  bool colok[G::SEGV];
  __device__ __forceinline__ void init(const WgradParams& p, int mbeg, int i0, int tid) {
    const int col = i0 + (tid % G::TPR) * G::SEGV * 8;
#pragma unroll
    for (int s = 0; s < G::SEGV; ++s) colok[s] = col + 8 * s < p.Nout;
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      m[i] = mbeg + tid / G::TPR + G::RSTEP * i;
      off[i] = (uint32_t)(m[i] * p.ldy + col) * (uint32_t)ESZ;
    }
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int mend, u32x4 (&d)[G::V],
                                       u32x4* d2 = nullptr) const {
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      const uint32_t base = m[i] < mend ? off[i] : HCB_OOB;
#pragma unroll
      for (int s = 0; s < G::SEGV; ++s) {
        const uint32_t o = colok[s] ? base + 16u * ESZ / 2 * s : HCB_OOB;
        d[i * G::SEGV + s] = buf_load16(r, o);
        if constexpr (ESZ == 4) d2[i * G::SEGV + s] = buf_load16(r, o + 16u);
      }
    }
  }
  __device__ __forceinline__ void advance(uint32_t step_bytes) {
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      off[i] += step_bytes;
      m[i] += ROWS;
    }
  }
};

// X operand (implicit im2col): rows m, columns j = (r, s, c) in [j0, j0 + COLS); the thread's
// segment lies in one tap, so its (dh, dw, c) are constant over the k-loop
template <int ROWS, int COLS, int NT, int ESZ = 2>
struct WgBLoad {
  using G = WgSeg<ROWS, COLS, NT>;
  int hh[G::RPT], ww[G::RPT], m[G::RPT];
  int off[G::RPT];  // byte offset of (n, hh, ww, c); meaningful only while in range
  int dh, dw;
  bool colok[G::SEGV];
  __device__ __forceinline__ void init(const WgradParams& p, int mbeg, int j0, int tid) {
    const int col = j0 + (tid % G::TPR) * G::SEGV * 8;
#pragma unroll
    for (int s = 0; s < G::SEGV; ++s) colok[s] = col + 8 * s < p.K;
    const int tap = col / p.C, c = col - tap * p.C;
    const int r = tap / p.S, s = tap - r * p.S;
    dh = r * p.dil_h - p.pad_h;
    dw = s * p.dil_w - p.pad_w;
    const int PQ = p.P * p.Q;
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      m[i] = mbeg + tid / G::TPR + G::RSTEP * i;
      const int n = m[i] / PQ, rem = m[i] - n * PQ, pp = rem / p.Q, qq = rem - pp * p.Q;
      hh[i] = pp * p.stride_h + dh;
      ww[i] = qq * p.stride_w + dw;
      off[i] = (((n * p.H + hh[i]) * p.W + ww[i]) * p.ldx + c) * ESZ;
    }
  }
  __device__ __forceinline__ void load(const WgradParams& p, __amdgpu_buffer_rsrc_t r, int mend,
                                       u32x4 (&d)[G::V], u32x4* d2 = nullptr) const {
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      const bool ok = m[i] < mend && (unsigned)hh[i] < (unsigned)p.H && (unsigned)ww[i] < (unsigned)p.W;
      const uint32_t base = ok ? (uint32_t)off[i] : HCB_OOB;
#pragma unroll
      for (int s = 0; s < G::SEGV; ++s) {
        const uint32_t o = colok[s] ? base + 16u * ESZ / 2 * s : HCB_OOB;
        d[i * G::SEGV + s] = buf_load16(r, o);
        if constexpr (ESZ == 4) d2[i * G::SEGV + s] = buf_load16(r, o + 16u);
      }
    }
  }
  __device__ __forceinline__ void advance(const WgAdvance& a, int sh) {
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      int w = ww[i] + a.dqw, h = hh[i], o = off[i] + a.dqo;
      const bool cq = w >= a.qs + dw;  // q wrapped: next output row
      w = cq ? w - a.qs : w;
      h = cq ? h + sh : h;
      o = cq ? o + a.qco : o;
      h += a.dph;
      o += a.dpo;
      const bool cp = h >= a.ps + dh;  // p wrapped: next image
      h = cp ? h - a.ps : h;
      o = cp ? o + a.pco : o;
      ww[i] = w;
      hh[i] = h;
      off[i] = o + a.dno;
      m[i] += ROWS;
    }
  }
};

// Shared-row variant of the X loader, for tiles whose columns all lie in ONE filter tap
// (1x1 convs, or C % tile cols == 0): every lane of a pixel row then needs the same source
// pixel, so instead of each lane stepping all RPT of its rows (VPR lanes redundantly per row),
// lane t of a wave steps just wave row t and the loads fetch their row's byte offset from the
// owning lane with one ds_bpermute (__shfl) + the lane's channel offset.
template <int ROWS, int COLS, int NT, int ESZ = 2>
struct WgBLoadShared {
  using G = WgSeg<ROWS, COLS, NT>;
  static constexpr int RW = 64 / G::TPR;   // rows per load instruction per wave
  static constexpr int TRK = RW * G::RPT;  // rows a wave loads per k-step
  static_assert(64 % G::TPR == 0 && TRK <= 64, "one tracked row per lane");
  int th, tw, tm, toff;  // tracked row: input row / col (tap applied), pixel index, byte offset
  int dh, dw;
  int src[G::RPT];       // lane owning row (lane / TPR) + RW * i of this wave
  uint32_t lane_c;       // this lane's byte offset within the row segment
  bool colok;
  __device__ __forceinline__ void init(const WgradParams& p, int mbeg, int j0, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int col = j0 + (tid % G::TPR) * 8;
    colok = col < p.K;
    lane_c = (uint32_t)((tid % G::TPR) * 8 * ESZ);
    const int tap = j0 / p.C, c0 = j0 - tap * p.C;  // the tile's tap (uniform)
    const int r = tap / p.S, s = tap - r * p.S;
    dh = r * p.dil_h - p.pad_h;
    dw = s * p.dil_w - p.pad_w;
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) src[i] = lane / G::TPR + RW * i;
    const int t = lane < TRK ? lane : TRK - 1;
    const int row = w * RW + t % RW + G::RSTEP * (t / RW);
    tm = mbeg + row;
    const int PQ = p.P * p.Q;
    const int n = tm / PQ, rem = tm - n * PQ, pp = rem / p.Q, qq = rem - pp * p.Q;
    th = pp * p.stride_h + dh;
    tw = qq * p.stride_w + dw;
    toff = (((n * p.H + th) * p.W + tw) * p.ldx + c0) * ESZ;
  }
  __device__ __forceinline__ void load(const WgradParams& p, __amdgpu_buffer_rsrc_t r, int mend,
                                       u32x4 (&d)[G::V], u32x4* d2 = nullptr) const {
    const bool ok = tm < mend && (unsigned)th < (unsigned)p.H && (unsigned)tw < (unsigned)p.W;
    const int val = ok ? toff : (int)HCB_OOB;
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      const uint32_t o = (uint32_t)__shfl(val, src[i], 64);  // OOB + lane_c stays out of range
      const uint32_t oo = colok ? o + lane_c : HCB_OOB;
      d[i] = buf_load16(r, oo);
      if constexpr (ESZ == 4) d2[i] = buf_load16(r, oo + 16u);
    }
  }
  __device__ __forceinline__ void advance(const WgAdvance& a, int sh) {
    int w = tw + a.dqw, h = th, o = toff + a.dqo;
    const bool cq = w >= a.qs + dw;
    w = cq ? w - a.qs : w;
    h = cq ? h + sh : h;
    o = cq ? o + a.qco : o;
    h += a.dph;
    o += a.dpo;
    const bool cp = h >= a.ps + dh;
    th = cp ? h - a.ps : h;
    tw = w;
    toff = (cp ? o + a.pco : o) + a.dno;
    tm += ROWS;
  }
};

// RIS: the X loader shares rows across lanes (every column of a tile in one filter tap), else
// per-lane rows. (16-bit operands; fp32 runs on the plane GEMMs, conv_p3_wgrad.h.)
template <int WM, int WN, int TM, int TN, bool RIS>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradParams p) {
  constexpr int BM = WM * TM, BN = WN * TN, BK = 64;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AVR = BM / 8, BVR = BN / 8;        // 16-byte vectors per LDS row
  constexpr int AV = BK * AVR / 256, BV = BK * BVR / 256;  // vectors per thread
  constexpr int ESZ = 2;
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

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  using GA = WgSeg<BK, BM, 256>;
  using GB = WgSeg<BK, BN, 256>;
  static_assert(GA::V == AV && GB::V == BV, "loader mapping");
  WgALoad<BK, BM, 256, ESZ> ald;
  std::conditional_t<RIS, WgBLoadShared<BK, BN, 256, ESZ>, WgBLoad<BK, BN, 256, ESZ>> bld;
  const uint32_t a_step = (uint32_t)(BK * p.ldy * ESZ);
  ald.init(p, kt_begin * BK, i0, tid);
  bld.init(p, kt_begin * BK, j0, tid);
  const WgAdvance adv = wg_advance(p, BK, ESZ);

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

  auto mfma_kstep = [&](const char* Ab, const char* Bb) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      act16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int col = wm * TM + i * 16;
        short4v lo = tr_read_a(Ab, ks * 32 + 8 * g, col);
        short4v hi = tr_read_a(Ab, ks * 32 + 8 * g + 4, col);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(act16x8, t);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int col = wn * TN + j * 16;
        short4v lo = tr_read_b(Bb, ks * 32 + 8 * g, col);
        short4v hi = tr_read_b(Bb, ks * 32 + 8 * g + 4, col);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(act16x8, t);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };
  // Two register sets: the loads of k-step k+2 are issued while k-step k is multiplied and
  // k+1 is stored to LDS, so a load has two k-steps (not one) of MFMA time to land -- the
  // 64x64 tile's 8 MFMAs per wave and k-step are far shorter than an L2 round trip.
  u32x4 sa[2][AV], sb[2][BV];
  // rows past this split's range come back as zeros without memory traffic, so the loads
  // and stores of the pipeline tail need no conditions (straight-line k-loop)
  const int mend = min(kt_end * BK, p.M);
  auto ld = [&](auto set_c) {
    constexpr int S = decltype(set_c)::value;
    ald.load(dyr, mend, sa[S], nullptr);
    bld.load(p, xr, mend, sb[S], nullptr);
    ald.advance(a_step);
    bld.advance(adv, p.stride_h);
  };
  auto st = [&](auto set_c, int buf) {
    constexpr int S = decltype(set_c)::value;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int o = buf * BK * BM * 2 + GA::lds_off(tid, v / GA::SEGV, v % GA::SEGV);
      *reinterpret_cast<u32x4*>(As + o) = sa[S][v];
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int o = buf * BK * BN * 2 + GB::lds_off(tid, v / GB::SEGV, v % GB::SEGV);
      *reinterpret_cast<u32x4*>(Bs + o) = sb[S][v];
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  const int nks = kt_end - kt_begin;
  ld(I0{});
  ld(I1{});
  st(I0{}, 0);
  __syncthreads();
  auto kstep = [&](auto cur_c, int k) {
    constexpr int cur = decltype(cur_c)::value;
    ld(cur_c);  // k-step k + 2 into set `cur` (stored to LDS one k-step ago)
    mfma_kstep(As + cur * BK * BM * 2, Bs + cur * BK * BN * 2);
    st(std::integral_constant<int, cur ^ 1>{}, cur ^ 1);  // k-step k + 1
    __syncthreads();
  };
  // an odd count runs one extra k-step over all-zero tiles (both operands out of range: adds
  // exactly 0) instead of a conditional second half, which made the compiler copy the
  // accumulators between register files every iteration
  for (int k = 0; k < nks; k += 2) {
    kstep(I0{}, k);
    kstep(I1{}, k + 1);
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
  wgrad_store_tile(p, Cs, LDC, BM, BN, i0, j0, tid, 256, gridDim.x == ntiles);
}

// ============================================================== LDS-DMA multi-stage variant
// Same GEMM, but both operands stream global -> LDS with buffer_load ... lds (no register
// staging) into an NST-deep ring, with counted s_waitcnt vmcnt + raw s_barrier keeping NST-2
// stages in flight (the conv_igemm_glds scheme). Each wave instruction fills RPI whole LDS rows
// (1 KiB); a lane fetches the GLOBAL 16-byte chunk that the swizzled transpose read expects at
// its LDS position (the 32-byte-slot XOR is an involution, applied to the source chunk). Wave
// tiles up to 64x64 halve the LDS bytes read per MFMA against the 32x32 register-staged
// kernel, which is LDS-read bound.
template <int N>
__device__ __forceinline__ void wg_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WM, int WN, int TM, int TN, int NST, bool CBIG>
__global__ __launch_bounds__(WM * WN * 64) void conv_wgrad_glds_kernel(WgradParams p) {
  constexpr int BM = WM * TM, BN = WN * TN, BK = 64;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NW = WM * WN;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;        // 16-byte chunks per LDS row
  constexpr int ARPI = 64 / ACPR, BRPI = 64 / BCPR;  // LDS rows filled by one wave instruction
  constexpr int AI = BK / ARPI / NW, BI = BK / BRPI / NW;  // instructions per wave per stage
  constexpr int LOADS = AI + BI;
  constexpr int STAGE = BK * (BM + BN) * 2;
  static_assert(AI * ARPI * NW == BK && BI * BRPI * NW == BK && AI >= 1 && BI >= 1, "tile / wave mapping");
  static_assert(NST >= 2 && NST <= 5 && LOADS * (NST - 2) <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
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
  const int kt_end = min(kt_begin + p.ksteps_per_split, nkt);
  if (kt_begin >= kt_end) return;  // uniform per workgroup

  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(p.dy, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);

  // per instruction v: this lane's LDS row within the stage and the global column it fetches
  int a_row[AI], a_col[AI];
#pragma unroll
  for (int v = 0; v < AI; ++v) {
    const int row = (wid * AI + v) * ARPI + lane / ACPR, pos = lane % ACPR;
    const int chunk = (((pos >> 1) ^ wg_swz<BM / 16>(row)) << 1) | (pos & 1);
    a_row[v] = row;
    a_col[v] = i0 + chunk * 8;
  }
  int b_row[BI], b_c[BI], b_dh[BI], b_dw[BI];
  bool b_ok[BI];
#pragma unroll
  for (int v = 0; v < BI; ++v) {
    const int row = (wid * BI + v) * BRPI + lane / BCPR, pos = lane % BCPR;
    const int chunk = (((pos >> 1) ^ wg_swz<BN / 16>(row)) << 1) | (pos & 1);
    const int col = j0 + chunk * 8;
    int tap, c;
    if constexpr (CBIG) {
      tap = j0 / p.C;
      c = j0 - tap * p.C + chunk * 8;
    } else {
      tap = (int)fdiv((uint32_t)col, p.fd_c);
      c = col - tap * p.C;
    }
    const int r = (int)fdiv((uint32_t)tap, p.fd_s), s = tap - r * p.S;
    b_row[v] = row;
    b_c[v] = c;
    b_dh[v] = r * p.dil_h - p.pad_h;
    b_dw[v] = s * p.dil_w - p.pad_w;
    b_ok[v] = col < p.K;
  }

  auto issue = [&](int stage, int kt) {
    const int mb = kt * BK;
    char* sA = smem + stage * STAGE;
    char* sB = sA + BK * BM * 2;
#pragma unroll
    for (int v = 0; v < AI; ++v) {
      const int m = mb + a_row[v];
      const uint32_t off = (a_col[v] < p.Nout && m < p.M) ? (uint32_t)(m * p.ldy + a_col[v]) * 2u : HCB_OOB;
      glds16(dyr, sA + (wid * AI + v) * ARPI * BM * 2, off);
    }
#pragma unroll
    for (int v = 0; v < BI; ++v) {
      const int m = mb + b_row[v];
      uint32_t off = HCB_OOB;
      if (b_ok[v] && m < p.M) {
        const int n = (int)fdiv((uint32_t)m, p.fd_pq);
        const int rem = m - n * p.P * p.Q;
        const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
        const int qq = rem - pp * p.Q;
        const int h = pp * p.stride_h + b_dh[v], w = qq * p.stride_w + b_dw[v];
        if ((unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W)
          off = (uint32_t)(((n * p.H + h) * p.W + w) * p.ldx + b_c[v]) * 2u;
      }
      glds16(xr, sB + (wid * BI + v) * BRPI * BN * 2, off);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads (lane supplies row + q4, columns col + 4*p4), swizzled slots
  const int li = lane & 15, g = lane >> 4, q4 = li >> 2, p4 = li & 3;
  auto tr_read_a = [&](const char* base, int row, int col) -> short4v {
    const int rr = row + q4, cb = (col + 4 * p4) * 2;
    const int slot = (cb >> 5) ^ wg_swz<BM / 16>(rr);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * BM * 2 + slot * 32 + (cb & 31)));
  };
  auto tr_read_b = [&](const char* base, int row, int col) -> short4v {
    const int rr = row + q4, cb = (col + 4 * p4) * 2;
    const int slot = (cb >> 5) ^ wg_swz<BN / 16>(rr);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * BN * 2 + slot * 32 + (cb & 31)));
  };

  const int nk = kt_end - kt_begin;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, kt_begin + s);
  for (int k = 0; k < nk; ++k) {
    // stage k has landed for this thread once at most min(NST-2, nk-1-k) later stages are
    // outstanding; the barrier then publishes every thread's DMA
    const int ahead = min(NST - 2, nk - 1 - k);
    if (ahead >= 3)
      wg_wait_vmcnt<(NST >= 5 ? 3 : 0) * LOADS>();
    else if (ahead == 2)
      wg_wait_vmcnt<(NST >= 4 ? 2 : 0) * LOADS>();
    else if (ahead == 1)
      wg_wait_vmcnt<LOADS>();
    else
      wg_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + NST - 1 < nk) issue((k + NST - 1) % NST, kt_begin + k + NST - 1);
    const char* Ab = smem + (k % NST) * STAGE;
    const char* Bb = Ab + BK * BM * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      act16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int col = wm * TM + i * 16;
        short4v lo = tr_read_a(Ab, ks * 32 + 8 * g, col);
        short4v hi = tr_read_a(Ab, ks * 32 + 8 * g + 4, col);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(act16x8, t);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = wn * TN + j * 16;
        short4v lo = tr_read_b(Bb, ks * 32 + 8 * g, col);
        short4v hi = tr_read_b(Bb, ks * 32 + 8 * g + 4, col);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(act16x8, t);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }
  __syncthreads();  // every wave is done with the ring before the epilogue reuses LDS

  constexpr int LDC = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * TM + i * 16 + g * 4 + e;
        const int col = wn * TN + j * 16 + li;
        Cs[row * LDC + col] = acc[i][j][e];
      }
  __syncthreads();
  wgrad_store_tile(p, Cs, LDC, BM, BN, i0, j0, tid, NW * 64, gridDim.x == ntiles);
}

// ============================================================== intra-workgroup split-K variant
// 4 waves, each with a 64x64 wave tile: WMt x WNt waves tile the output block and KS waves
// share each (BM x BN) block, splitting every 128-deep k-step (128 / KS rows each); their
// partial tiles are summed through LDS at the end. <1,1,4>: every wave owns the whole 64x64
// tile over a 32-deep quarter -- against the 2x2 arrangement of 32x32 wave tiles this halves
// the transposed LDS fragment bytes per MFMA (16 reads feed 16 MFMAs per wave, not 8 reads 4
// MFMAs), and that kernel is LDS-read bound. <2,1,2> / <1,2,2>: 128x64 / 64x128 blocks.
// RIS: X loader with rows shared across lanes (one filter tap per tile), else per-lane rows
template <int WMt, int WNt, int KS, bool RIS>
__global__ __launch_bounds__(256) void conv_wgrad_kq_kernel(WgradParams p) {
  static_assert(WMt * WNt * KS == 4, "4 waves");
  constexpr int BM = 64 * WMt, BN = 64 * WNt, BK = 128, KW = BK / KS;  // KW: k rows per wave
  constexpr int AVR = BM / 8, BVR = BN / 8;                // 16-byte vectors per LDS row
  constexpr int AV = BK * AVR / 256, BV = BK * BVR / 256;  // vectors per thread per k-step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;                    // [2][BK][BM] bf16
  char* Bs = smem + 2 * BK * BM * 2;  // [2][BK][BN]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid % KS, wmn = wid / KS;  // k share, output sub-tile
  const int wm = wmn / WNt, wn = wmn % WNt;
  const int tiles_m = (p.Nout + BM - 1) / BM;
  const int tiles_n = (p.K + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int i0 = tm * BM, j0 = tn * BN;

  // this split's pixel rows (the host plans splits in 64-row units)
  const int mbeg = split * p.ksteps_per_split * 64;
  const int mend = min(mbeg + p.ksteps_per_split * 64, p.M);
  if (mbeg >= mend) return;  // uniform per workgroup
  const int nk = (mend - mbeg + BK - 1) / BK;

  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(p.dy, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  u32x4 ra[AV], rb[BV];
  using GA = WgSeg<BK, BM, 256>;
  using GB = WgSeg<BK, BN, 256>;
  static_assert(GA::V == AV && GB::V == BV, "loader mapping");
  WgALoad<BK, BM, 256> ald;
  std::conditional_t<RIS, WgBLoadShared<BK, BN, 256>, WgBLoad<BK, BN, 256>> bld;
  const uint32_t a_step = (uint32_t)(BK * p.ldy * 2);
  ald.init(p, mbeg, i0, tid);
  bld.init(p, mbeg, j0, tid);
  const WgAdvance adv = wg_advance(p, BK);
  auto gload = [&]() {  // k-steps in order: the loaders hold the next k-step's rows
    ald.load(dyr, mend, ra);
    bld.load(p, xr, mend, rb);
    ald.advance(a_step);
    bld.advance(adv, p.stride_h);
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v)
      *reinterpret_cast<u32x4*>(As + buf * BK * BM * 2 + GA::lds_off(tid, v / GA::SEGV, v % GA::SEGV)) = ra[v];
#pragma unroll
    for (int v = 0; v < BV; ++v)
      *reinterpret_cast<u32x4*>(Bs + buf * BK * BN * 2 + GB::lds_off(tid, v / GB::SEGV, v % GB::SEGV)) = rb[v];
  };

  const int li = lane & 15, g = lane >> 4, q4 = li >> 2, p4 = li & 3;
  auto tr_read_a = [&](const char* base, int row, int col) -> short4v {
    const int rr = row + q4, cb = (col + 4 * p4) * 2;
    const int slot = (cb >> 5) ^ wg_swz<BM / 16>(rr);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * BM * 2 + slot * 32 + (cb & 31)));
  };
  auto tr_read_b = [&](const char* base, int row, int col) -> short4v {
    const int rr = row + q4, cb = (col + 4 * p4) * 2;
    const int slot = (cb >> 5) ^ wg_swz<BN / 16>(rr);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * BN * 2 + slot * 32 + (cb & 31)));
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfma_kstep = [&](const char* Ab, const char* Bb) {
#pragma unroll
    for (int ks = 0; ks < KW / 32; ++ks) {
      const int krow = wk * KW + ks * 32;
      act16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        short4v lo = tr_read_a(Ab, krow + 8 * g, wm * 64 + i * 16);
        short4v hi = tr_read_a(Ab, krow + 8 * g + 4, wm * 64 + i * 16);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(act16x8, t);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        short4v lo = tr_read_b(Bb, krow + 8 * g, wn * 64 + j * 16);
        short4v hi = tr_read_b(Bb, krow + 8 * g + 4, wn * 64 + j * 16);
        short8 t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(act16x8, t);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };

  // the 64x64 (1,1,4) variant keeps the single-set loop: with two sets the compiler copies its 64
  // accumulators between register files every k-step (56 extra VALU per two k-steps)
  constexpr bool PIPE2 = !(WMt == 1 && WNt == 1);
  if constexpr (PIPE2) {
    // two register sets, k-step k + 2 in flight while k is multiplied (see conv_wgrad_kernel)
    u32x4 sa[2][AV], sb[2][BV];
    auto ld = [&](auto set_c) {
      constexpr int S = decltype(set_c)::value;
      ald.load(dyr, mend, sa[S]);
      bld.load(p, xr, mend, sb[S]);
      ald.advance(a_step);
      bld.advance(adv, p.stride_h);
    };
    auto st = [&](auto set_c, int buf) {
      constexpr int S = decltype(set_c)::value;
#pragma unroll
      for (int v = 0; v < AV; ++v)
        *reinterpret_cast<u32x4*>(As + buf * BK * BM * 2 + GA::lds_off(tid, v / GA::SEGV, v % GA::SEGV)) = sa[S][v];
#pragma unroll
      for (int v = 0; v < BV; ++v)
        *reinterpret_cast<u32x4*>(Bs + buf * BK * BN * 2 + GB::lds_off(tid, v / GB::SEGV, v % GB::SEGV)) = sb[S][v];
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    ld(I0{});
    ld(I1{});
    st(I0{}, 0);
    __syncthreads();
    auto kstep = [&](auto cur_c) {
      constexpr int cur = decltype(cur_c)::value;
      ld(cur_c);
      mfma_kstep(As + cur * BK * BM * 2, Bs + cur * BK * BN * 2);
      st(std::integral_constant<int, cur ^ 1>{}, cur ^ 1);
      __syncthreads();
    };
    for (int k = 0; k < nk; k += 2) {  // odd counts: one extra all-zero k-step (adds 0)
      kstep(I0{});
      kstep(I1{});
    }
  } else {
    gload();
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload();
      mfma_kstep(As + cur * BK * BM * 2, Bs + cur * BK * BN * 2);
      if (kt + 1 < nk) lstore(cur ^ 1);
      __syncthreads();
    }
  }

  // the KS k-shares' partial tiles -> LDS, summed, then stored / atomically added
  constexpr int LDC = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);  // [KS][BM][LDC]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wk * BM + wm * 64 + i * 16 + g * 4 + e) * LDC + wn * 64 + j * 16 + li] = acc[i][j][e];
  __syncthreads();
  if constexpr (KS > 1) {
    for (int idx = tid; idx < BM * BN; idx += 256) {
      const int row = idx / BN, col = idx - row * BN;
      float v = Cs[row * LDC + col];
#pragma unroll
      for (int k = 1; k < KS; ++k) v += Cs[(k * BM + row) * LDC + col];
      Cs[row * LDC + col] = v;
    }
    __syncthreads();
  }
  wgrad_store_tile(p, Cs, LDC, BM, BN, i0, j0, tid, 256, gridDim.x == ntiles);
}

// every column tile of width BN lies in one filter tap (shared-row X loader)
static bool wgrad_one_tap(const WgradParams& p, int BN) { return p.R * p.S == 1 || (p.C % BN) == 0; }

template <int WMt, int WNt, int KS>
static void wlaunch_kq(const WgradParams& p, int splits, hipStream_t st) {
  constexpr int BM = 64 * WMt, BN = 64 * WNt;
  const int tiles = ((p.Nout + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  const size_t lds_main = (size_t)2 * 128 * (BM + BN) * 2;
  const size_t lds_epi = (size_t)KS * BM * (BN + 4) * 4;
  const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)conv_wgrad_kq_kernel<WMt, WNt, KS, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)conv_wgrad_kq_kernel<WMt, WNt, KS, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  const dim3 grid(tiles * splits);
  if (wgrad_one_tap(p, BN))
    hipLaunchKernelGGL((conv_wgrad_kq_kernel<WMt, WNt, KS, true>), grid, dim3(256), lds, st, p);
  else
    hipLaunchKernelGGL((conv_wgrad_kq_kernel<WMt, WNt, KS, false>), grid, dim3(256), lds, st, p);
}

template <int WM, int WN, int TM, int TN, int NST>
static void wlaunch_glds(const WgradParams& p, int splits, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  const int tiles = ((p.Nout + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  const size_t lds_main = (size_t)NST * 64 * (BM + BN) * 2;
  const size_t lds_epi = (size_t)BM * (BN + 4) * 4;
  const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)conv_wgrad_glds_kernel<WM, WN, TM, TN, NST, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)conv_wgrad_glds_kernel<WM, WN, TM, TN, NST, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  dim3 grid(tiles * splits);
  if ((p.C % BN) == 0)
    hipLaunchKernelGGL((conv_wgrad_glds_kernel<WM, WN, TM, TN, NST, true>), grid, dim3(WM * WN * 64), lds, st, p);
  else
    hipLaunchKernelGGL((conv_wgrad_glds_kernel<WM, WN, TM, TN, NST, false>), grid, dim3(WM * WN * 64), lds, st, p);
}

template <int WM, int WN, int TM, int TN>
static void wlaunch(const WgradParams& p, int splits, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  int tiles = ((p.Nout + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  size_t lds_main = (size_t)2 * 64 * (BM + BN) * 2;
  size_t lds_epi = (size_t)BM * (BN + 4) * 4;
  size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  dim3 grid(tiles * splits);
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)conv_wgrad_kernel<WM, WN, TM, TN, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)conv_wgrad_kernel<WM, WN, TM, TN, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  if (wgrad_one_tap(p, BN))
    hipLaunchKernelGGL((conv_wgrad_kernel<WM, WN, TM, TN, true>), grid, dim3(256), lds, st, p);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<WM, WN, TM, TN, false>), grid, dim3(256), lds, st, p);
}

// cfg 0..2: register-staged {128x128, 64x128, 64x64}; 3..9: LDS-DMA ring {128x128 (4 waves of
// 64x64, NST 4), 128x128 (8 waves of 64x32), 256x128 (8 waves of 64x64), 128x256 (8 waves of
// 64x64), 64x128 (8 waves of 32x32, NST 4), 64x64 (4 waves, NST 4), 64x128 (4 waves of 64x32,
// NST 4)}
// 10-12: intra-workgroup k-split 64x64, 128x64, 64x128; 13-14: register-staged 128x64 / 64x128 with
// 64x32 / 32x64 wave tiles (twice the MFMAs per loaded row of the 64x64 tile)
constexpr int N_WGRAD_CFG = 15;
int wgrad_tile_m(int cfg) {
  static const int t[N_WGRAD_CFG] = {128, 64, 64, 128, 128, 256, 128, 64, 64, 64, 64, 128, 64, 128, 64};
  return (cfg >= 0 && cfg < N_WGRAD_CFG) ? t[cfg] : 64;
}
int wgrad_tile_n(int cfg) {
  static const int t[N_WGRAD_CFG] = {128, 128, 64, 128, 128, 128, 256, 128, 64, 128, 64, 64, 128, 64, 128};
  return (cfg >= 0 && cfg < N_WGRAD_CFG) ? t[cfg] : 64;
}

void launch_conv_wgrad(const WgradParams& p, int cfg, int splits, hipStream_t st) {
  // the register-staged loaders keep a thread's 16-byte vector inside one filter tap (every
  // weight pack already requires C % 8 == 0; bindings.cpp checks it)
  switch (cfg) {
    case 0: wlaunch<2, 2, 64, 64>(p, splits, st); break;  // 128 x 128
    case 1: wlaunch<1, 4, 64, 32>(p, splits, st); break;  // 64 x 128
    case 3: wlaunch_glds<2, 2, 64, 64, 4>(p, splits, st); break;
    case 4: wlaunch_glds<2, 4, 64, 32, 3>(p, splits, st); break;
    case 5: wlaunch_glds<4, 2, 64, 64, 3>(p, splits, st); break;
    case 6: wlaunch_glds<2, 4, 64, 64, 3>(p, splits, st); break;
    case 7: wlaunch_glds<2, 4, 32, 32, 4>(p, splits, st); break;
    case 8: wlaunch_glds<2, 2, 32, 32, 4>(p, splits, st); break;
    case 9: wlaunch_glds<1, 4, 64, 32, 4>(p, splits, st); break;
    case 10: wlaunch_kq<1, 1, 4>(p, splits, st); break;
    case 11: wlaunch_kq<2, 1, 2>(p, splits, st); break;
    case 12: wlaunch_kq<1, 2, 2>(p, splits, st); break;
    case 13: wlaunch<2, 2, 64, 32>(p, splits, st); break;  // 128 x 64
    case 14: wlaunch<2, 2, 32, 64>(p, splits, st); break;  // 64 x 128
    default: wlaunch<2, 2, 32, 32>(p, splits, st); break; // 64 x 64
  }
}

}  // namespace hcb
