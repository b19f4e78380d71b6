// Forward / data-gradient plane GEMM (bf16x6 on hi / mid / lo planes): the kernel template and its
// launchers (instantiated in conv_p3.hip; the weight-gradient kernel, conv_p3_wgrad.h, shares the
// fragment helpers).
#pragma once
#include "common.h"
#include "igemm_epilogue.h"
#include "igemm_loader.h"
#include "kernels.h"

namespace hcb {

// Tile geometry of the plane GEMMs. KW: channels per ring slot (k-depth): 64 (128-byte LDS rows, the
// bf16 kernels' layout) or 32 (64-byte rows: half the LDS per slot, so a 128x128 or 256x128 block
// tile fits a 3- or 2-slot ring and each loaded byte feeds twice the MFMAs of a 64x128 tile -- the
// per-CU L2 -> LDS fill rate, not the MFMA, is what bounds the smaller tiles).
template <int KW>
__device__ __forceinline__ int p3_swz(int row) {
  // 16-byte chunk XOR per row, conflict-free ds_read_b128 fragment reads: 128-byte rows: the
  // generic kernels' (row >> 1) & 7; 64-byte rows: (row >> 2) & 2 (each lane group of the read
  // then covers the 16 distinct 16-byte bank quads of a 256-byte bank row)
  if constexpr (KW == 64) return (row >> 1) & 7;
  else return (row >> 2) & 2;
}

// the fragments of one slot (KS = KW / 32 halves of 32, three planes of each operand) in registers
constexpr int NPL = 3;
template <int TM, int TN, int KS>
struct P3Frags {
  static constexpr int MI = TM / 16, NI = TN / 16;
  u32x4 a[KS][NPL][MI], b[KS][NPL][NI];
};

// every fragment read of the slot (LDS -> registers), issued back to back
template <int WM, int WN, int TM, int TN, int KW>
__device__ __forceinline__ void p3_read(const u32x4* A, const u32x4* B, P3Frags<TM, TN, KW / 32>& f, int wm, int wn,
                                        int lane) {
  constexpr int MI = TM / 16, NI = TN / 16, BM = WM * TM, BN = WN * TN, CPR = KW / 8;
  constexpr int AIMG = BM * CPR, BIMG = BN * CPR;  // one plane image, in u32x4
  const int frow = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < KW / 32; ++ks) {
    const int ch = ks * 4 + fq;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * TM + i * 16 + frow, o = row * CPR + (ch ^ p3_swz<KW>(row));
#pragma unroll
      for (int t = 0; t < NPL; ++t) f.a[ks][t][i] = A[t * AIMG + o];
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wn * TN + j * 16 + frow, o = row * CPR + (ch ^ p3_swz<KW>(row));
#pragma unroll
      for (int t = 0; t < NPL; ++t) f.b[ks][t][j] = B[t * BIMG + o];
    }
  }
}

// the KS x MI x NI x 6 MFMAs of the slot on register fragments (small terms first)
template <int TM, int TN, int KS>
__device__ __forceinline__ void p3_mma(const P3Frags<TM, TN, KS>& f, f32x4 (&acc)[TM / 16][TN / 16]) {
  constexpr int MI = TM / 16, NI = TN / 16;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        acc[i][j] = mfma_bf16(f.a[ks][2][i], f.b[ks][0][j], acc[i][j]);
        acc[i][j] = mfma_bf16(f.a[ks][0][i], f.b[ks][2][j], acc[i][j]);
        acc[i][j] = mfma_bf16(f.a[ks][1][i], f.b[ks][1][j], acc[i][j]);
        acc[i][j] = mfma_bf16(f.a[ks][1][i], f.b[ks][0][j], acc[i][j]);
        acc[i][j] = mfma_bf16(f.a[ks][0][i], f.b[ks][1][j], acc[i][j]);
        acc[i][j] = mfma_bf16(f.a[ks][0][i], f.b[ks][0][j], acc[i][j]);
      }
}

template <int BM, int BN, int KW>
constexpr size_t p3_stage_bytes() {
  return (size_t)NPL * (BM + BN) * KW * 2;
}
// LDS offset of the fused BN-backward parameters: above the ring and the epilogue staging
template <int BM, int BN, int WM, int KW, int NST>
constexpr size_t p3_param_off() {
  const size_t a = NST * p3_stage_bytes<BM, BN, KW>(), b = igemm_epilogue_lds(BM, BN, WM);
  return a > b ? a : b;
}
// data-grad GEMMs with at most this many 64-deep k-steps fetch their fused BN-backward epilogue
// operands before the main loop
constexpr int EARLY_EPI_KSTEPS_P3 = 2;

// ============================================================== forward / data gradient
// x: three bf16 planes of the NHWC input, p.x_plane bytes apart (each plane p.x_bytes long);
// w / w_lo / w_lo2: the hi / mid / lo weight packs [Nout][Kpad]. NST-slot LDS-DMA ring of KW-deep
// slots with EARLY RELEASE: a slot is refilled as soon as every wave holds its fragments in
// registers, not after the MFMAs, so NST slots of DMA are in flight during a slot's MFMAs; the
// refill issues (and the next slot's fragment reads) are interleaved with the slot's MFMAs
// (igemm_loader.h ilv_schedule). Split-K: a tile's S shares meet through splitk_gather.
// BNB: the fused BN-backward epilogue (data gradient producing a BN layer's dy: ReLU gating from the
// hi plane of y or from z, sum(g) / sum(g * xhat) into p.bnb_acc), fp32 z / beta source / output
// OCC: workgroups per CU the tile is built for (2: <= 80 KB of LDS and <= 512 / (2 * waves per SIMD)
// registers per wave, so one workgroup's barrier / DMA waits are covered by the other's MFMAs)
template <int OCC, int NW>
constexpr int p3_regs_per_wave() {
  return 512 / (OCC * NW / 4 > 0 ? OCC * NW / 4 : 1);
}
template <int WM, int WN, int TM, int TN, int KW, int NST, bool CBIG, bool LHSDIL, bool BNB, int OCC = 1>
__global__ __launch_bounds__(WM* WN * 64, OCC* WM* WN / 4) void conv_igemm_p3_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NT = WM * WN * 64, CPR = KW / 8, RB = KW * 2;  // threads; chunks and bytes per LDS row
  constexpr int RP = NT / CPR;                                    // tile rows per load pass
  constexpr int AV = BM / RP, BV = BN / RP;
  constexpr int LOADS = NPL * (AV + BV);  // LDS-DMA instructions per thread per slot
  constexpr int AIMG = BM * RB, BIMG = BN * RB;
  constexpr int STAGE = (int)p3_stage_bytes<BM, BN, KW>();
  static_assert(AV * RP == BM && BV * RP == BN, "tile rows must be a multiple of the load pass");
  static_assert(LOADS * (NST - 1) <= 63 && NST >= 2 && NST <= 4, "vmcnt range");
  static_assert(p3_param_off<BM, BN, WM, KW, NST>() + bnb_param_lds(BN) <= 160 * 1024,
                "ring + BN parameters must fit LDS");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // a tile's splits are neighbours: same XCD
  const int nk_all = p.Kpad / KW;
  const int parts = p.splits, tile = bid / parts, part = bid - tile * parts;
  const int kb = part * nk_all / parts, nk = (part + 1) * nk_all / parts - kb;  // this share's k-slots
  // lane-linear LDS image (row tid / CPR of the pass, position tid % CPR); the lane fetches the
  // GLOBAL chunk the swizzled read expects there (the XOR is an involution; RP * v and a wave's
  // row base are multiples of 16, so the row's swizzle is a function of tid)
  const int chunk = (tid % CPR) ^ p3_swz<KW>(tid / CPR);

  const char* xb = reinterpret_cast<const char*>(p.x);
  const __amdgpu_buffer_rsrc_t xr0 = make_rsrc(xb, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr1 = make_rsrc(xb + p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr2 = make_rsrc(xb + 2 * (size_t)p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr0 = make_rsrc(p.w, p.w_bytes);
  const __amdgpu_buffer_rsrc_t wr1 = make_rsrc(p.w_lo, p.w_bytes);
  const __amdgpu_buffer_rsrc_t wr2 = make_rsrc(p.w_lo2, p.w_bytes);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  ALoader<AV, CBIG, LHSDIL, RP, 2, KW> al;
  al.init(p, m0, tid, chunk);
  uint32_t b_off[BV];
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const int j = n0 + tid / CPR + RP * v;
    b_off[v] = (j < p.Nout) ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
  }
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int WROWS = 64 / CPR;  // LDS rows one wave instruction fills
  // every slot issue is made, also past the share's last k-slot (kl >= nk: all offsets out of range,
  // the pieces land zeros in a slot nobody reads again), so the vmcnt arithmetic is uniform and the
  // issue sits in the same basic block as the MFMAs it is interleaved with
  auto issue = [&](int stage, int kl) {
    const int kt = kb + kl;
    const bool live = kl < nk;
    uint32_t off[AV];
    al.offsets(p, kt, chunk, off);  // k-steps are issued strictly in order
    char* sa = smem + stage * STAGE + wid * WROWS * RB;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      if (!live) off[v] = HCB_OOB;
      glds16(xr0, sa + RP * v * RB, off[v]);
      glds16(xr1, sa + AIMG + RP * v * RB, off[v]);
      glds16(xr2, sa + 2 * AIMG + RP * v * RB, off[v]);
    }
    char* sb = smem + stage * STAGE + NPL * AIMG + wid * WROWS * RB;
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const uint32_t o = (b_off[v] == HCB_OOB || !live) ? HCB_OOB : b_off[v] + (uint32_t)kt * (uint32_t)RB;
      glds16(wr0, sb + RP * v * RB, o);
      glds16(wr1, sb + BIMG + RP * v * RB, o);
      glds16(wr2, sb + 2 * BIMG + RP * v * RB, o);
    }
  };
  if (kb > 0) al.seek(p, kb);
  EpiPrefetch<WM, WN, TM, TN, BNB, true> pre;
  pre.load_shift(p, n0, wn, lane);
  constexpr size_t PARAM_OFF = p3_param_off<BM, BN, WM, KW, NST>();
  if constexpr (BNB) stage_bnb_params<BN, NT>(p, n0, smem + PARAM_OFF);  // published by the first barrier
  const bool early = BNB && parts == 1 && nk * KW <= EARLY_EPI_KSTEPS_P3 * 64;
  if (early) pre.load(p, 0, m0, n0, tid);
#pragma unroll
  for (int s = 0; s < NST; ++s) issue(s, s);
  // wait until at most `ahead` later slots' DMA is outstanding for this thread
  auto wait_ahead = [&](auto ahead_c) {
    constexpr int ahead = decltype(ahead_c)::value;
    wait_vmcnt<ahead * LOADS>();
  };
  auto read = [&](int k, P3Frags<TM, TN, KW / 32>& f) {
    const char* sb = smem + (k % NST) * STAGE;
    p3_read<WM, WN, TM, TN, KW>(reinterpret_cast<const u32x4*>(sb), reinterpret_cast<const u32x4*>(sb + NPL * AIMG), f,
                                wm, wn, lane);
  };
  // two register fragment sets when they fit (PIPE): slot k+1's fragment reads are in flight
  // while slot k's MFMAs run, and ONE barrier per slot both publishes slot k+1's DMA and retires
  // every wave's reads of slot k (which is refilled right after it); otherwise one set, read,
  // then a second barrier before the refill
  constexpr int FREGS = (MI + NI) * NPL * 4 * (KW / 32), AREGS = MI * NI * 4;
  constexpr int RBUDGET = p3_regs_per_wave<OCC, WM * WN>() - 56 < 400 ? p3_regs_per_wave<OCC, WM * WN>() - 56 : 400;
  constexpr bool PIPE = 2 * FREGS + AREGS <= RBUDGET && !(BNB && RBUDGET < 400);
  constexpr int NMF = (KW / 32) * MI * NI * 6, NRD = (KW / 32) * (MI + NI) * NPL;
  if constexpr (PIPE) {
    // slot k+1 has landed for this thread once at most the NST - 2 slots after it are outstanding
    P3Frags<TM, TN, KW / 32> fr[2];
    wait_ahead(std::integral_constant<int, NST - 1>{});
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, fr[0]);
    auto body = [&](int k, P3Frags<TM, TN, KW / 32>& cur, P3Frags<TM, TN, KW / 32>& nxt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot k are done
      wait_ahead(std::integral_constant<int, NST - 2>{});  // slot k+1 landed for this thread
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(k % NST, k + NST);
      read(k + 1, nxt);
      p3_mma<TM, TN, KW / 32>(cur, acc);
      ilv_schedule<NMF, LOADS, NRD>();
    };
    for (int k = 0; k < nk; k += 2) {
      body(k, fr[0], fr[1]);
      if (k + 1 < nk) body(k + 1, fr[1], fr[0]);
    }
  } else {
    P3Frags<TM, TN, KW / 32> fr;
    for (int kt = 0; kt < nk; ++kt) {
      // slot kt has landed for this thread once at most the later slots' loads are outstanding;
      // the barrier publishes every thread's DMA
      wait_ahead(std::integral_constant<int, NST - 1>{});
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(kt, fr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot are done
      __builtin_amdgcn_s_barrier();                        // ... and every other wave's
      asm volatile("" ::: "memory");
      issue(kt % NST, kt + NST);
      p3_mma<TM, TN, KW / 32>(fr, acc);
      ilv_schedule<NMF, LOADS, 0>();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy pieces have landed before LDS reuse
  __syncthreads();  // every wave is done reading the ring before the epilogue reuses LDS
  if (parts > 1 && !splitk_gather<MI, NI, NT>(p, acc, smem, tile, part, parts, tid)) return;
  igemm_epilogue<WM, WN, TM, TN, BNB, true>(p, acc, smem, tm, m0, n0, wm, wn, lane, tid, pre, early,
                                            BNB ? smem + PARAM_OFF : nullptr);
}

template <typename K>
static void p3_set_lds_once(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int WM, int WN, int TM, int TN, int KW, int NST, bool BNB, int OCC = 1>
static void launch_p3(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN, NT = WM * WN * 64;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN) * p.splits;
  const size_t lds_main = (size_t)NST * p3_stage_bytes<BM, BN, KW>();  // dummy refills use every slot
  const size_t lds_epi = igemm_epilogue_lds(BM, BN, WM);
  size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  if (BNB) lds = p3_param_off<BM, BN, WM, KW, NST>() + bnb_param_lds(BN);
  const bool cbig = (p.C % 64) == 0;
  const bool lhs = p.idil_h > 1 || p.idil_w > 1;
  static bool once = false;
  if (!once) {
    p3_set_lds_once(conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, true, false, BNB, OCC>);
    p3_set_lds_once(conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, true, true, BNB, OCC>);
    p3_set_lds_once(conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, false, false, BNB, OCC>);
    p3_set_lds_once(conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, false, true, BNB, OCC>);
    once = true;
  }
  if (cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, true, false, BNB, OCC>), dim3(tiles), dim3(NT),
                       lds, st, p);
  else if (cbig && lhs)
    hipLaunchKernelGGL((conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, true, true, BNB, OCC>), dim3(tiles), dim3(NT),
                       lds, st, p);
  else if (!cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, false, false, BNB, OCC>), dim3(tiles), dim3(NT),
                       lds, st, p);
  else
    hipLaunchKernelGGL((conv_igemm_p3_kernel<WM, WN, TM, TN, KW, NST, false, true, BNB, OCC>), dim3(tiles), dim3(NT),
                       lds, st, p);
}

// p3 cfg (block tile, waves x wave tile, slot depth, ring slots):
//   64-deep slots, 2 slots:  0 128x64 (2x2 of 64x32), 1 64x128 (2x2 of 32x64), 2 128x64 (4x2 of 32x32),
//                            3 64x128 (2x4 of 32x32), 4 64x64 (2x2 of 32x32), 5 128x64 (4x1 of 32x64),
//                            6 64x128 (1x4 of 64x32)
//   32-deep slots:           7 128x128 (2x4 of 64x32, 3 slots), 8 128x128 (4x2 of 32x64, 3 slots),
//                            9 128x128 (2x2 of 64x64, 3 slots), 10 256x128 (4x2 of 64x64, 2 slots),
//                            11 128x256 (2x4 of 64x64, 2 slots), 12 64x128 (2x2 of 32x64, 4 slots),
//                            13 128x64 (2x2 of 64x32, 4 slots)
//   32-deep, two per CU:     14 128x64 (2x2 of 64x32, 2 slots), 15 64x128 (2x2 of 32x64, 2 slots),
//                            16 64x64 (2x2 of 32x32, 3 slots)
//   32-deep, three per CU:   17 64x64 (2x2 of 32x32, 2 slots)
template <bool BNB>
static void launch_p3_cfg(const ConvParams& p, int cfg, hipStream_t st) {
  switch (cfg) {
    case 1: launch_p3<2, 2, 32, 64, 64, 2, BNB, 1>(p, st); break;
    case 2: launch_p3<4, 2, 32, 32, 64, 2, BNB, 1>(p, st); break;
    case 3: launch_p3<2, 4, 32, 32, 64, 2, BNB, 1>(p, st); break;
    case 4: launch_p3<2, 2, 32, 32, 64, 2, BNB, 1>(p, st); break;
    case 5: launch_p3<4, 1, 32, 64, 64, 2, BNB, 1>(p, st); break;
    case 6: launch_p3<1, 4, 64, 32, 64, 2, BNB, 1>(p, st); break;
    case 7: launch_p3<2, 4, 64, 32, 32, 3, BNB, 1>(p, st); break;
    case 8: launch_p3<4, 2, 32, 64, 32, 3, BNB, 1>(p, st); break;
    case 9: launch_p3<2, 2, 64, 64, 32, 3, BNB, 1>(p, st); break;
    case 10: launch_p3<4, 2, 64, 64, 32, 2, BNB, 1>(p, st); break;
    case 11: launch_p3<2, 4, 64, 64, 32, 2, BNB, 1>(p, st); break;
    case 12: launch_p3<2, 2, 32, 64, 32, 4, BNB, 1>(p, st); break;
    case 13: launch_p3<2, 2, 64, 32, 32, 4, BNB, 1>(p, st); break;
    case 14: launch_p3<2, 2, 64, 32, 32, 2, BNB, 2>(p, st); break;
    case 15: launch_p3<2, 2, 32, 64, 32, 2, BNB, 2>(p, st); break;
    case 16: launch_p3<2, 2, 32, 32, 32, 3, BNB, 2>(p, st); break;
    case 17: launch_p3<2, 2, 32, 32, 32, 2, BNB, 3>(p, st); break;
    default: launch_p3<2, 2, 64, 32, 64, 2, BNB, 1>(p, st); break;
  }
}

}  // namespace hcb
