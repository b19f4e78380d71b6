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
//   * im2col is never materialised: each lane gathers 16-byte channel vectors of the input
//     with raw buffer loads; halo / padding / tail rows use an out-of-range offset, which
//     the buffer unit turns into zeros (no branches around loads).
//   * two main loops, picked per layer by the autotuner:
//       - "reg":  register-staged double-buffered LDS, one barrier per k-step;
//       - "glds": LDS-DMA (buffer_load ... lds) straight into an NST-deep ring of LDS
//         stages, counted s_waitcnt vmcnt + raw s_barrier so NST-2 stages stay in flight
//         across barriers (the latency lever at ~1-2 workgroups per CU). The LDS image is
//         lane-linear; the XOR swizzle is applied to the per-lane SOURCE chunk and to the
//         fragment reads (same involution), per the gfx950 glds rules.
//   * LDS rows are 128 B (BK=64 bf16); 16-byte chunks are XOR-swizzled with (row>>1)&7 so
//     the ds_read_b128 fragment reads are bank-conflict free.
//   * XCD-aware block remap so neighbouring tiles (sharing the im2col panel) sit on one
//     XCD's L2.
//   * epilogue (igemm_epilogue.h): fused per-channel BatchNorm statistics from the
//     accumulators, LDS-staged fully coalesced 16-byte stores, beta-accumulate, bias,
//     fp32 output, strided-output remap.
#include "common.h"
#include "igemm_epilogue.h"
#include "igemm_loader.h"
#include "kernels.h"

namespace hcb {

// data-grad GEMMs with at most this many 64-deep k-steps issue their fused BN-backward
// epilogue loads before the main loop (EpiPrefetch)
constexpr int EARLY_EPI_KSTEPS = 2;

// LDS offset of the fused BN-backward parameters: above the main-loop buffers and the epilogue
// staging (full ring for the LDS-DMA kernels)
constexpr size_t reg_param_off(int BM, int BN, int WM) {
  const size_t a = (size_t)2 * (BM + BN) * 8 * 16, b = igemm_epilogue_lds(BM, BN, WM);
  return a > b ? a : b;
}
constexpr size_t glds_param_off(int BM, int BN, int WM, int NST) {
  const size_t a = (size_t)NST * (BM + BN) * 128, b = igemm_epilogue_lds(BM, BN, WM);
  return a > b ? a : b;
}

// SCHED: issue every fragment read of the 64-deep k-step (both 32-deep halves) before the first
// MFMA, behind a scheduling barrier, so the second half's LDS reads overlap the first half's MFMAs
// (the compiler otherwise interleaves one read per MFMA group with an lgkmcnt wait on it, exposing
// the LDS latency MI times per half). On for the LDS-DMA and patch kernels (3-8% on the 3x3
// layers, +0.7% step after a retune); measured neutral on the register-staged kernels, whose
// prefetch registers it competes with, so off there (profiles/r3k_patch_sched_retune.txt).
template <int WM, int WN, int TM, int TN, bool SCHED = false>
__device__ __forceinline__ void mfma_tile_step(const u32x4* Ab, const u32x4* Bb, f32x4 (&acc)[TM / 16][TN / 16],
                                               int wm, int wn, int lane) {
  constexpr int MI = TM / 16, NI = TN / 16;
  const int frow = lane & 15, fq = lane >> 4;
  if constexpr (SCHED) {
  act16x8 af[2][MI], bfr[2][NI];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int ch = ks * 4 + fq;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * TM + i * 16 + frow;
      af[ks][i] = __builtin_bit_cast(act16x8, Ab[row * 8 + (ch ^ ((row >> 1) & 7))]);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wn * TN + j * 16 + frow;
      bfr[ks][j] = __builtin_bit_cast(act16x8, Bb[row * 8 + (ch ^ ((row >> 1) & 7))]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(af[ks][i], bfr[ks][j], acc[i][j]);
  } else {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    act16x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      int row = wm * TM + i * 16 + frow;
      int ch = ks * 4 + fq;
      af[i] = __builtin_bit_cast(act16x8, Ab[row * 8 + (ch ^ ((row >> 1) & 7))]);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int row = wn * TN + j * 16 + frow;
      int ch = ks * 4 + fq;
      bfr[j] = __builtin_bit_cast(act16x8, Bb[row * 8 + (ch ^ ((row >> 1) & 7))]);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  }
  }
}

// ============================================================== register-staged main loop
// (16-bit operands; fp32 runs on the plane GEMMs, conv_p3.hip)
template <int WM, int WN, int TM, int TN, bool CBIG, bool LHSDIL, bool BNB>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN, BK = 64;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AV = BM / 32, BV = BN / 32;  // 16-byte vectors per thread per k-step
  static_assert(WM * WN == 4, "4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int NB = p.Kpad > 64 ? 2 : 1;  // LDS buffers (one for a single k-step)
  u32x4* As = reinterpret_cast<u32x4*>(smem);  // [NB][BM*8]
  u32x4* Bs = As + NB * BM * 8;                 // [NB][BN*8]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int chunk = tid & 7;

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  ALoader<AV, CBIG, LHSDIL, 32, 2> al;
  al.init(p, m0, tid, chunk);
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

  auto gload = [&](int kt) {
    uint32_t off[AV];
    al.offsets(p, kt, chunk, off);
#pragma unroll
    for (int v = 0; v < AV; ++v) ra[v] = buf_load16(xr, off[v]);
#pragma unroll
    for (int v = 0; v < BV; ++v) rb[v] = buf_load16(wr, b_off[v] == HCB_OOB ? HCB_OOB : b_off[v] + (uint32_t)kt * 128u);
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int row = (tid >> 3) + 32 * v;
      As[buf * BM * 8 + row * 8 + (chunk ^ ((row >> 1) & 7))] = ra[v];
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int row = (tid >> 3) + 32 * v;
      Bs[buf * BN * 8 + row * 8 + (chunk ^ ((row >> 1) & 7))] = rb[v];
    }
  };

  const int nk = p.Kpad / BK;
  EpiPrefetch<WM, WN, TM, TN, BNB> pre;
  pre.load_shift(p, n0, wn, lane);
  constexpr size_t PARAM_OFF = reg_param_off(BM, BN, WM);
  if constexpr (BNB) stage_bnb_params<BN, 256>(p, n0, smem + PARAM_OFF);  // published by the first barrier
  const bool early = BNB && nk <= EARLY_EPI_KSTEPS;
  if (early) pre.load(p, 0, m0, n0, tid);
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    mfma_tile_step<WM, WN, TM, TN, false>(As + cur * BM * 8, Bs + cur * BN * 8, acc, wm, wn, lane);
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }
  igemm_epilogue<WM, WN, TM, TN, BNB>(p, acc, smem, tm, m0, n0, wm, wn, lane, tid, pre, early, smem + PARAM_OFF);
}

// ============================================================== LDS-DMA multi-stage main loop
// NST-stage ring of 64-deep k-steps, NST - 1 in flight; the refill of step k + NST - 1 is issued
// right after the barrier of step k. (Spreading that refill among step k's MFMAs -- the plane GEMMs'
// ilv_schedule, +1.4% fp32 -- measured neutral here: bf16 9,698-9,704 vs 9,707-9,728 img/s,
// profiles/r5_prune_variants.txt; the register-pipelined, two-k-step and occupancy-ring variants of
// this loop were removed in round 5 for the same reason.)
template <int WM, int WN, int TM, int TN, int NST, bool CBIG, bool LHSDIL, bool BNB>
__global__ __launch_bounds__(WM * WN * 64, WM * WN / 4) void conv_igemm_glds_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NT = WM * WN * 64, RP = NT / 8;  // threads; tile rows per load pass
  constexpr int AV = BM / RP, BV = BN / RP;
  constexpr int LOADS = AV + BV;                // LDS-DMA instructions per thread per stage
  constexpr int STAGE = (BM + BN) * 128;        // one k-step's A + B image
  static_assert((WM * WN == 4 || WM * WN == 8) && NST >= 2 && NST <= 6, "config");
  static_assert(AV * RP == BM && BV * RP == BN, "tile rows must be a multiple of the load pass");
  static_assert(LOADS * (NST - 2) <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // a tile's splits are neighbours: same XCD
  const int S = p.splits;
  const int tile = bid / S, split = bid - tile * S;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // lane-linear LDS image: lane -> (row = (tid>>3)+RP*v, position tid&7); the lane fetches the
  // GLOBAL chunk that the swizzled read expects at that position (involution; RP*v and the
  // wave's 8-row base are multiples of 16, so (row>>1)&7 == (tid>>4)&7).
  const int chunk = (tid & 7) ^ ((tid >> 4) & 7);

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, p.w_bytes);
  ALoader<AV, CBIG, LHSDIL, RP> al;
  al.init(p, m0, tid, chunk);
  uint32_t b_off[BV];
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    int j = n0 + (tid >> 3) + RP * v;
    b_off[v] = (j < p.Nout) ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
  }
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = p.Kpad / 64;
  const int kb = split * nk_all / S, nk = (split + 1) * nk_all / S - kb;  // this block's k-steps
  auto issue = [&](int stage, int kl) {
    const bool live = kl < nk;
    const int kt = kb + kl;
    uint32_t off[AV];
    al.offsets(p, kt, chunk, off);  // k-steps are issued strictly in order
    char* sbase = smem + stage * STAGE;
#pragma unroll
    for (int v = 0; v < AV; ++v) glds16(xr, sbase + (wid * 8 + RP * v) * 128, live ? off[v] : HCB_OOB);
#pragma unroll
    for (int v = 0; v < BV; ++v)
      glds16(wr, sbase + BM * 128 + (wid * 8 + RP * v) * 128,
             (!live || b_off[v] == HCB_OOB) ? HCB_OOB : b_off[v] + (uint32_t)kt * 128u);
  };
  if (kb > 0) al.seek(p, kb);
  EpiPrefetch<WM, WN, TM, TN, BNB> pre;
  pre.load_shift(p, n0, wn, lane);
  constexpr size_t PARAM_OFF = glds_param_off(BM, BN, WM, NST);
  constexpr bool PARAM_LDS = PARAM_OFF + bnb_param_lds(BN) <= 160 * 1024;
  if constexpr (BNB && PARAM_LDS) stage_bnb_params<BN, NT>(p, n0, smem + PARAM_OFF);  // published by the first barrier
  const bool early = BNB && S == 1 && nk <= EARLY_EPI_KSTEPS;
  if (early) pre.load(p, 0, m0, n0, tid);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed for this thread once at most min(NST-2, nk-1-kt) later stages
    // are still outstanding; the barrier then publishes every thread's DMA.
    const int ahead = min(NST - 2, nk - 1 - kt);
    if (ahead >= 4)
      wait_vmcnt<(NST >= 6 ? 4 : 0) * LOADS>();
    else if (ahead == 3)
      wait_vmcnt<(NST >= 5 ? 3 : 0) * LOADS>();
    else if (ahead == 2)
      wait_vmcnt<(NST >= 4 ? 2 : 0) * LOADS>();
    else if (ahead == 1)
      wait_vmcnt<LOADS>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) issue((kt + NST - 1) % NST, kt + NST - 1);
    const char* sb = smem + (kt % NST) * STAGE;
    mfma_tile_step<WM, WN, TM, TN, true>(reinterpret_cast<const u32x4*>(sb),
                                         reinterpret_cast<const u32x4*>(sb + BM * 128), acc, wm, wn, lane);
  }
  __syncthreads();  // every wave is done reading the ring before the epilogue reuses LDS
  if (S > 1 && !splitk_gather<MI, NI, NT>(p, acc, smem, tile, split, S, tid)) return;
  igemm_epilogue<WM, WN, TM, TN, BNB>(p, acc, smem, tm, m0, n0, wm, wn, lane, tid, pre, early,
                                      PARAM_LDS ? smem + PARAM_OFF : nullptr);
}

// ============================================================== launch
// One instantiation per (im2col path, lhs-dilation, fused BN-backward epilogue); the BNB
// variants are separate kernels so the plain ones keep their register budget.
template <typename K>
static void set_lds_once(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int WM, int WN, int TM, int TN, bool BNB>
static void launch_reg(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  int tiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN);
  // a single k-step (1x1 over <= 64 channels) uses one buffer pair
  size_t lds_main = (size_t)(p.Kpad > 64 ? 2 : 1) * (BM + BN) * 8 * 16;
  size_t lds_epi = igemm_epilogue_lds(BM, BN, WM, igemm_stage16(p));
  size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  if (BNB) lds = reg_param_off(BM, BN, WM) + bnb_param_lds(BN);
  bool cbig = (p.C % 64) == 0;
  bool lhs = p.idil_h > 1 || p.idil_w > 1;
  static bool once = false;
  if (!once) {
    set_lds_once(conv_igemm_kernel<WM, WN, TM, TN, true, false, BNB>);
    set_lds_once(conv_igemm_kernel<WM, WN, TM, TN, true, true, BNB>);
    set_lds_once(conv_igemm_kernel<WM, WN, TM, TN, false, false, BNB>);
    set_lds_once(conv_igemm_kernel<WM, WN, TM, TN, false, true, BNB>);
    once = true;
  }
  if (cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, true, false, BNB>), dim3(tiles), dim3(256), lds, st, p);
  else if (cbig && lhs)
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, true, true, BNB>), dim3(tiles), dim3(256), lds, st, p);
  else if (!cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, false, false, BNB>), dim3(tiles), dim3(256), lds, st, p);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, TM, TN, false, true, BNB>), dim3(tiles), dim3(256), lds, st, p);
}

template <int WM, int WN, int TM, int TN, int NST, bool BNB>
static void launch_glds(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN, NT = WM * WN * 64;
  int tiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN) * p.splits;
  // a block never touches more ring stages than it has k-steps (short-K layers: 1x1 over 64-256
  // channels, 1-4 k-steps, get the LDS they use, so more workgroups fit per CU)
  const int ksteps = (p.Kpad / 64 + p.splits - 1) / p.splits;
  const int stages = ksteps < NST ? (ksteps > 0 ? ksteps : 1) : NST;
  size_t lds_main = (size_t)stages * (BM + BN) * 128;
  size_t lds_epi = igemm_epilogue_lds(BM, BN, WM, igemm_stage16(p));
  size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
  if (BNB && glds_param_off(BM, BN, WM, NST) + bnb_param_lds(BN) <= 160 * 1024)
    lds = glds_param_off(BM, BN, WM, NST) + bnb_param_lds(BN);
  bool cbig = (p.C % 64) == 0;
  bool lhs = p.idil_h > 1 || p.idil_w > 1;
  static bool once = false;
  if (!once) {
    set_lds_once(conv_igemm_glds_kernel<WM, WN, TM, TN, NST, true, false, BNB>);
    set_lds_once(conv_igemm_glds_kernel<WM, WN, TM, TN, NST, true, true, BNB>);
    set_lds_once(conv_igemm_glds_kernel<WM, WN, TM, TN, NST, false, false, BNB>);
    set_lds_once(conv_igemm_glds_kernel<WM, WN, TM, TN, NST, false, true, BNB>);
    once = true;
  }
  if (cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_glds_kernel<WM, WN, TM, TN, NST, true, false, BNB>), dim3(tiles), dim3(NT), lds, st, p);
  else if (cbig && lhs)
    hipLaunchKernelGGL((conv_igemm_glds_kernel<WM, WN, TM, TN, NST, true, true, BNB>), dim3(tiles), dim3(NT), lds, st, p);
  else if (!cbig && !lhs)
    hipLaunchKernelGGL((conv_igemm_glds_kernel<WM, WN, TM, TN, NST, false, false, BNB>), dim3(tiles), dim3(NT), lds, st,
                       p);
  else
    hipLaunchKernelGGL((conv_igemm_glds_kernel<WM, WN, TM, TN, NST, false, true, BNB>), dim3(tiles), dim3(NT), lds, st, p);
}

// cfg: 0..3 register-staged {128x128, 128x64, 64x64, 64x128}; 4..7 the same tiles on the
// LDS-DMA ring (NST 3, 3, 4, 3); 8..11 deeper rings for latency-bound few-tile layers
// (128x128 NST 4 and 5, 128x64 NST 6, 64x128 NST 6); 12..16 eight-wave workgroups (two
// waves per SIMD when a layer has only ~1 tile per CU): 128x128 as 2x4 waves of 64x32 and as
// 4x2 of 32x64, 256x128 (4x2 of 64x64), 128x256 (2x4 of 64x64), 64x128 (2x4 of 32x32);
// 17..21 the 3x3 patch kernels (conv3x3_patch.hip): 128x128, 256x128, 256x64, 128x64, 128x128;
// (round 5: the rejected variants -- two k-steps per stage, cfg 22-26; occupancy-sized two-slot
// rings, 27-30; the register-pipelined loop, 31-37; the plane kernel on one 16-bit plane, 100-117 --
// were measured without a step gain and removed: profiles/r5_prune_variants.txt)
constexpr int N_CONV_CFG = 22;
int conv_tile_m(int cfg) {
  static const int t[N_CONV_CFG] = {128, 128, 64, 64, 128, 128, 64, 64, 128, 128, 128,
                                    64,  128, 128, 256, 128, 64, 128, 256, 256, 128, 128};
  return (cfg >= 0 && cfg < N_CONV_CFG) ? t[cfg] : 128;
}
int conv_tile_n(int cfg) {
  static const int t[N_CONV_CFG] = {128, 64,  64,  128, 128, 64,  64, 128, 128, 128, 64,
                                    128, 128, 128, 128, 256, 128, 128, 128, 64, 64, 128};
  return (cfg >= 0 && cfg < N_CONV_CFG) ? t[cfg] : 128;
}

template <bool BNB>
static void launch_cfg(const ConvParams& p, int cfg, hipStream_t st) {
  switch (cfg) {
    case 0: launch_reg<2, 2, 64, 64, BNB>(p, st); break;    // 128 x 128
    case 1: launch_reg<4, 1, 32, 64, BNB>(p, st); break;    // 128 x 64
    case 2: launch_reg<2, 2, 32, 32, BNB>(p, st); break;    // 64 x 64
    case 3: launch_reg<1, 4, 64, 32, BNB>(p, st); break;    // 64 x 128
    case 4: launch_glds<2, 2, 64, 64, 3, BNB>(p, st); break;
    case 5: launch_glds<4, 1, 32, 64, 3, BNB>(p, st); break;
    case 6: launch_glds<2, 2, 32, 32, 4, BNB>(p, st); break;
    case 7: launch_glds<1, 4, 64, 32, 3, BNB>(p, st); break;
    case 8: launch_glds<2, 2, 64, 64, 4, BNB>(p, st); break;
    case 9: launch_glds<2, 2, 64, 64, 5, BNB>(p, st); break;
    case 10: launch_glds<4, 1, 32, 64, 6, BNB>(p, st); break;
    case 11: launch_glds<1, 4, 64, 32, 6, BNB>(p, st); break;
    case 12: launch_glds<2, 4, 64, 32, 3, BNB>(p, st); break;
    case 13: launch_glds<4, 2, 32, 64, 3, BNB>(p, st); break;
    case 14: launch_glds<4, 2, 64, 64, 3, BNB>(p, st); break;
    case 15: launch_glds<2, 4, 64, 64, 3, BNB>(p, st); break;
    case 16: launch_glds<2, 4, 32, 32, 4, BNB>(p, st); break;
    default: launch_reg<2, 2, 64, 64, BNB>(p, st); break;
  }
}

void launch_conv_igemm(const ConvParams& p, int cfg, hipStream_t st) {
  if (cfg >= CONV_PATCH_CFG0 && cfg < CONV_PATCH_CFG0 + 5) {
    if (launch_conv3x3_patch(p, cfg, st)) return;
    // not a 3x3 / stride-1 problem (or its patch does not fit LDS): an LDS-DMA kernel of the
    // same row tile (so per-tile statistics slabs keep their size), without split-K
    static const int fallback[5] = {13, 14, 14, 5, 13};
    ConvParams q = p;
    q.splits = 1;
    cfg = fallback[cfg - CONV_PATCH_CFG0];
    if (q.bnb_acc != nullptr)
      launch_cfg<true>(q, cfg, st);
    else
      launch_cfg<false>(q, cfg, st);
    return;
  }
  if (p.bnb_acc != nullptr)
    launch_cfg<true>(p, cfg, st);
  else
    launch_cfg<false>(p, cfg, st);
}

}  // namespace hcb
