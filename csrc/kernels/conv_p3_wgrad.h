// Weight-gradient plane GEMM (conv_wgrad_p3_kernel, fp32 on three bf16 planes) and its launcher,
// instantiated in conv_p3.hip.
#pragma once
#include "conv_p3_fwd.h"

namespace hcb {

// ============================================================== weight gradient
// dW[Nout][K] += sum_m dY[m][Nout] * im2col(X)[m][K] on planes: dy planes p.dy_plane bytes apart,
// x planes p.x_plane bytes apart. Both operands have the reduction index (pixels) as their outer
// dimension: staged as [64 pixels][tile cols] rows and read back transposed (ds_read_b64_tr_b16),
// 32-byte slots XOR-swizzled (wg_swz) as in conv_wgrad.hip. NST-deep LDS-DMA ring.
template <int NSLOT>
__device__ __forceinline__ int p3w_swz(int row) {
  if constexpr (NSLOT >= 8) return (row & 3) | ((row >> 1) & 4);
  else return ((row >> 1) & 1) | ((row >> 2) & 2);
}

// BK: pixel rows (reduction depth) per ring slot, 64 or 32 (32: half the LDS per slot, so 128x128 /
// 256x128 block tiles fit); NST slots with early release; PIPE (when two fragment sets fit the
// register budget): slot k+1's transposed fragment reads in flight during slot k's MFMAs, one
// barrier per slot. The refill issues are interleaved with the MFMAs (ilv_schedule).
template <int WM, int WN, int TM, int TN, int NST, int BK, bool CBIG, int OCC = 1>
__global__ __launch_bounds__(WM* WN * 64, OCC* WM* WN / 4) void conv_wgrad_p3_kernel(WgradParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16, KS = BK / 32;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;        // 16-byte chunks per LDS row
  constexpr int ARPI = 64 / ACPR, BRPI = 64 / BCPR;  // LDS rows filled by one wave instruction
  constexpr int AI = BK / ARPI / NW, BI = BK / BRPI / NW;  // instructions per wave per plane and slot
  constexpr int LOADS = NPL * (AI + BI);
  constexpr int AIMG = BK * BM * 2, BIMG = BK * BN * 2;
  constexpr int STAGE = NPL * (AIMG + BIMG);
  static_assert(AI * ARPI * NW == BK && BI * BRPI * NW == BK && AI >= 1 && BI >= 1, "tile / wave mapping");
  static_assert(NST >= 2 && NST <= 3 && LOADS * (NST - 1) <= 63 && NST * STAGE <= 160 * 1024, "ring");
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
  // the host plans splits in 64-row k-steps; this block's pixel rows [mbeg, mend)
  const int mbeg = split * p.ksteps_per_split * 64;
  const int mend = min(mbeg + p.ksteps_per_split * 64, p.M);
  if (mbeg >= mend) return;  // uniform per workgroup

  const char* db = reinterpret_cast<const char*>(p.dy);
  const char* xb = reinterpret_cast<const char*>(p.x);
  const __amdgpu_buffer_rsrc_t dyr0 = make_rsrc(db, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t dyr1 = make_rsrc(db + p.dy_plane, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t dyr2 = make_rsrc(db + 2 * (size_t)p.dy_plane, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr0 = make_rsrc(xb, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr1 = make_rsrc(xb + p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr2 = make_rsrc(xb + 2 * (size_t)p.x_plane, p.x_bytes);

  int a_row[AI], a_col[AI];
#pragma unroll
  for (int v = 0; v < AI; ++v) {
    const int row = (wid * AI + v) * ARPI + lane / ACPR, pos = lane % ACPR;
    const int chunk = (((pos >> 1) ^ p3w_swz<BM / 16>(row)) << 1) | (pos & 1);
    a_row[v] = row;
    a_col[v] = i0 + chunk * 8;
  }
  int b_row[BI], b_c[BI], b_dh[BI], b_dw[BI];
  bool b_ok[BI];
#pragma unroll
  for (int v = 0; v < BI; ++v) {
    const int row = (wid * BI + v) * BRPI + lane / BCPR, pos = lane % BCPR;
    const int chunk = (((pos >> 1) ^ p3w_swz<BN / 16>(row)) << 1) | (pos & 1);
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

  // every slot issue is made, also past the last k-step (rows >= mend read as zeros into a slot
  // nobody reads again), so the vmcnt arithmetic is uniform and the issue can be interleaved with
  // the MFMAs of the same basic block (igemm_loader.h ilv_schedule)
  auto issue = [&](int stage, int kl) {
    const int mb = mbeg + kl * BK;
    char* sA = smem + stage * STAGE;
    char* sB = sA + NPL * AIMG;
#pragma unroll
    for (int v = 0; v < AI; ++v) {
      const int m = mb + a_row[v];
      const bool ok = (a_col[v] < p.Nout) & (m < mend);
      const uint32_t off = ((uint32_t)(m * p.ldy + a_col[v]) * 2u) | ((uint32_t)!ok << 31);
      char* d = sA + (wid * AI + v) * ARPI * BM * 2;
      glds16(dyr0, d, off);
      glds16(dyr1, d + AIMG, off);
      glds16(dyr2, d + 2 * AIMG, off);
    }
#pragma unroll
    for (int v = 0; v < BI; ++v) {
      const int m = mb + b_row[v];
      // branch-free (a divergent branch here would split the slot's basic block and keep the
      // issue out of the MFMA interleave): every lane computes its offset, a select rejects it
      const int n = (int)fdiv((uint32_t)m, p.fd_pq);
      const int rem = m - n * p.P * p.Q;
      const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
      const int qq = rem - pp * p.Q;
      const int h = pp * p.stride_h + b_dh[v], w = qq * p.stride_w + b_dw[v];
      const bool ok = b_ok[v] & (m < mend) & ((unsigned)h < (unsigned)p.H) & ((unsigned)w < (unsigned)p.W);
      const uint32_t raw = (uint32_t)(((n * p.H + h) * p.W + w) * p.ldx + b_c[v]) * 2u;
      const uint32_t off = raw | ((uint32_t)!ok << 31);  // >= HCB_OOB: out of range
      char* d = sB + (wid * BI + v) * BRPI * BN * 2;
      glds16(xr0, d, off);
      glds16(xr1, d + BIMG, off);
      glds16(xr2, d + 2 * BIMG, off);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads (lane supplies row + q4, columns col + 4*p4), swizzled slots
  const int li = lane & 15, g = lane >> 4, q4 = li >> 2, p4 = li & 3;
  auto frag = [&](const char* base, int ncols, int krow, int col) -> u32x4 {
    short4v v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rr = krow + 4 * h + q4, cb = (col + 4 * p4) * 2;
      const int sw = ncols == BM ? p3w_swz<BM / 16>(rr) : p3w_swz<BN / 16>(rr);
      const int slot = (cb >> 5) ^ sw;
      v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4v HCB_LDS*)(base + rr * ncols * 2 + slot * 32 + (cb & 31)));
    }
    short8 t = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
    return __builtin_bit_cast(u32x4, t);
  };
  using Fr = P3Frags<TM, TN, KS>;
  auto read = [&](int k, Fr& f) {
    const char* Ab = smem + (k % NST) * STAGE;
    const char* Bb = Ab + NPL * AIMG;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int t = 0; t < NPL; ++t) f.a[ks][t][i] = frag(Ab + t * AIMG, BM, ks * 32 + 8 * g, wm * TM + i * 16);
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int t = 0; t < NPL; ++t) f.b[ks][t][j] = frag(Bb + t * BIMG, BN, ks * 32 + 8 * g, wn * TN + j * 16);
    }
  };

  const int nk = (mend - mbeg + BK - 1) / BK;
  // every slot issue is made, also past the last k-step (its rows read as zeros), so slot k has
  // landed for this thread once at most the NST - 1 (PIPE: slot k+1 once NST - 2) slots after it are
  // outstanding
#pragma unroll
  for (int s = 0; s < NST; ++s) issue(s, s);
  constexpr int FREGS = (MI + NI) * NPL * 4 * KS, AREGS = MI * NI * 4;
  constexpr int RBUDGET = p3_regs_per_wave<OCC, WM * WN>() - 88 < 400 ? p3_regs_per_wave<OCC, WM * WN>() - 88 : 400;
  constexpr bool PIPE = 2 * FREGS + AREGS <= RBUDGET;
  constexpr int NMF = KS * MI * NI * 6, NRD = 2 * KS * (MI + NI) * NPL;
  if constexpr (PIPE) {
    Fr fr[2];
    wait_vmcnt<(NST - 1) * LOADS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, fr[0]);
    auto body = [&](int k, Fr& cur, Fr& nxt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot k are done
      wait_vmcnt<(NST - 2) * LOADS>();                     // slot k+1 landed for this thread
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(k % NST, k + NST);
      read(k + 1, nxt);
      p3_mma<TM, TN, KS>(cur, acc);
      ilv_schedule<NMF, LOADS, NRD>();
    };
    for (int k = 0; k < nk; k += 2) {
      body(k, fr[0], fr[1]);
      if (k + 1 < nk) body(k + 1, fr[1], fr[0]);
    }
  } else {
    Fr fr;
    for (int k = 0; k < nk; ++k) {
      wait_vmcnt<(NST - 1) * LOADS>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(k, fr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot are done
      __builtin_amdgcn_s_barrier();                        // ... and every other wave's
      asm volatile("" ::: "memory");
      issue(k % NST, k + NST);
      p3_mma<TM, TN, KS>(fr, acc);
      ilv_schedule<NMF, LOADS, 0>();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy pieces have landed before LDS reuse
  __syncthreads();  // every wave is done with the ring before the epilogue reuses LDS

  constexpr int LDC = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wm * TM + i * 16 + g * 4 + e) * LDC + wn * TN + j * 16 + li] = acc[i][j][e];
  __syncthreads();
  const bool sole = gridDim.x == ntiles;
  for (int idx = tid; idx < BM * BN; idx += NT) {
    const int row = idx / BN, col = idx - row * BN;
    const int gi = i0 + row, gj = j0 + col;
    if (gi < p.Nout && gj < p.K) {
      float* d = p.dw + (size_t)gi * p.K + gj;
      if (sole)
        *d += Cs[row * LDC + col];
      else
        atomicAdd(d, Cs[row * LDC + col]);
    }
  }
}

template <int WM, int WN, int TM, int TN, int NST, int BK, int OCC = 1>
static void wlaunch_p3(const WgradParams& p, int splits, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  const int tiles = ((p.Nout + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  const size_t lds_main = (size_t)NST * NPL * BK * (BM + BN) * 2;
  const size_t lds_epi = (size_t)BM * (BN + 4) * 4;
  const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  static bool once = false;
  if (!once) {
    p3_set_lds_once(conv_wgrad_p3_kernel<WM, WN, TM, TN, NST, BK, true, OCC>);
    p3_set_lds_once(conv_wgrad_p3_kernel<WM, WN, TM, TN, NST, BK, false, OCC>);
    once = true;
  }
  const dim3 grid(tiles * splits);
  if ((p.C % BN) == 0)
    hipLaunchKernelGGL((conv_wgrad_p3_kernel<WM, WN, TM, TN, NST, BK, true, OCC>), grid, dim3(WM * WN * 64), lds, st, p);
  else
    hipLaunchKernelGGL((conv_wgrad_p3_kernel<WM, WN, TM, TN, NST, BK, false, OCC>), grid, dim3(WM * WN * 64), lds, st, p);
}

}  // namespace hcb
