// 3x3 / stride 1 / pad 1 convolutions with the input patch RESIDENT IN LDS (gfx950 MFMA,
// v_mfma_f32_16x16x32_bf16, NHWC bf16). Serves the ResNet bottleneck conv2 forward and its data
// gradient (a stride-1 3x3 conv of dy with the flipped weights), i.e. the 3x3 Conv2D fwd /
// bwd-data primitives of the reference's MKL-DNN path (driven by
// /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81).
//
// Why a separate kernel: the generic implicit GEMM (conv_igemm.hip) fetches an im2col A tile per
// filter tap, so every input pixel crosses L2 -> LDS nine times. The ResNet-50 3x3 layers run
// at ~8 TB/s of aggregate L2 -> CU traffic (the per-CU fetch rate, not the MFMAs, sets their
// time: profiles/r2h_pmc_conv_classes.txt, MFMA busy 14-18%). Here a block's BM consecutive
// output pixels map to ONE contiguous range of the zero-padded input (padded linear index
// Lp(n, p, q) = n*(H+2)*(W+2) + p*(W+2) + q; tap (r, s) reads Lp + r*(W+2) + s), so the block
// loads that range once per 64-channel slab -- ~BM + 2*(W+2) rows instead of 9*BM -- and reads
// the nine shifted A operands straight out of it. Only the weight tile streams per k-step.
//
//   * k-steps run slab-major, tap-minor: step g = (slab g/9, tap g%9); the weight tiles stream
//     through an NST-deep LDS-DMA ring (buffer_load ... lds, counted vmcnt, raw s_barrier) as in
//     conv_igemm_glds_kernel;
//   * the patch is double buffered: the next slab's patch is issued (LDS-DMA, halo rows with an
//     out-of-range offset -> zeros, no memory traffic) inside the group of tap NST-1 of the
//     current slab, the first step at which no wave can still be reading that buffer; the vmcnt
//     of every step counts the patch loads of the groups in flight exactly;
//   * LDS rows are 128 B (64 channels), the 16-byte chunks XOR-swizzled with (row>>1)&7 on the
//     source side (the DMA image is lane-linear) and on the fragment reads;
//   * split-K over channel slabs (splitk_gather) and the shared epilogue (fused BN statistics,
//     fused BN-backward for data gradients) as in the generic kernels.
#include "common.h"
#include "igemm_epilogue.h"
#include "kernels.h"

namespace hcb {

// s_waitcnt vmcnt with a wave-uniform run-time count (the immediate is chosen by a branch)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
#define HCB_VMW(k)                                     \
  case k:                                              \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
  switch (n) {
    HCB_VMW(0) HCB_VMW(1) HCB_VMW(2) HCB_VMW(3) HCB_VMW(4) HCB_VMW(5) HCB_VMW(6) HCB_VMW(7)
    HCB_VMW(8) HCB_VMW(9) HCB_VMW(10) HCB_VMW(11) HCB_VMW(12) HCB_VMW(13) HCB_VMW(14) HCB_VMW(15)
    HCB_VMW(16) HCB_VMW(17) HCB_VMW(18) HCB_VMW(19) HCB_VMW(20) HCB_VMW(21) HCB_VMW(22) HCB_VMW(23)
    HCB_VMW(24) HCB_VMW(25) HCB_VMW(26) HCB_VMW(27) HCB_VMW(28) HCB_VMW(29) HCB_VMW(30) HCB_VMW(31)
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef HCB_VMW
}

// padded linear index of output pixel m (P == H, Q == W)
__device__ __forceinline__ int patch_lp(const ConvParams& p, int m) {
  const int n = (int)fdiv((uint32_t)m, p.fd_hw), r = m - n * p.H * p.W;
  const int pp = (int)fdiv((uint32_t)r, p.fd_w), qq = r - pp * p.W;
  return (n * (p.H + 2) + pp) * (p.W + 2) + qq;
}

// Fragment reads: 16-byte XOR-swizzled ds_read_b128 as in the generic kernels. The patch rows a
// fragment reads start at an arbitrary row (the tap offset), so a b128 lane group (lanes 0-3,12-15
// of one k-chunk column and 4-11 of the next) can meet 2-way bank conflicts (32-39% extra LDS
// cycles measured); a conflict-free form with two ds_read_b64 per fragment (each column's halves
// read in opposite order) was measured slower -- twice the LDS instructions cost more than the
// conflicts (profiles/r3k_patch_sched_retune.txt, variant b128 vs main).
__device__ __forceinline__ u32x4 frag_read(const u32x4* base, int row, int ch) {
  return base[row * 8 + (ch ^ ((row >> 1) & 7))];
}

// every fragment read of the step first, then the MFMAs (see conv_igemm.hip mfma_tile_step SCHED)
template <int WM, int WN, int TM, int TN>
__device__ __forceinline__ void mfma_patch_step(const u32x4* Pb, const u32x4* Bb, const int (&prow)[TM / 16], int tapoff,
                                                f32x4 (&acc)[TM / 16][TN / 16], int wn, int lane) {
  constexpr int MI = TM / 16, NI = TN / 16;
  const int frow = lane & 15, fq = lane >> 4;
  act16x8 af[2][MI], bfr[2][NI];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int ch = ks * 4 + fq;
#pragma unroll
    for (int i = 0; i < MI; ++i) af[ks][i] = __builtin_bit_cast(act16x8, frag_read(Pb, prow[i] + tapoff, ch));
#pragma unroll
    for (int j = 0; j < NI; ++j) bfr[ks][j] = __builtin_bit_cast(act16x8, frag_read(Bb, wn * TN + j * 16 + frow, ch));
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(af[ks][i], bfr[ks][j], acc[i][j]);
}

// LDS bytes of the main loop / the BN-backward parameter offset, shared by kernel and launcher.
// The patch is double buffered only when some block reduces more than one 64-channel slab (a
// single-slab problem -- the stage-1 3x3 layers over 64 channels -- keeps one buffer: half the
// patch LDS, more workgroups per CU).
__host__ __device__ inline int patch_buffers(const ConvParams& p) { return p.C / 64 > p.splits ? 2 : 1; }
template <int BM, int BN, int WM, int NST>
__host__ __device__ inline size_t patch_main_lds(const ConvParams& p) {
  return (size_t)NST * BN * 128 + (size_t)patch_buffers(p) * p.patch_rows * 128;
}
template <int BM, int BN, int WM, int NST>
__host__ __device__ inline size_t patch_param_off(const ConvParams& p) {
  const size_t a = patch_main_lds<BM, BN, WM, NST>(p), b = igemm_epilogue_lds(BM, BN, WM);
  return a > b ? a : b;
}

template <int WM, int WN, int TM, int TN, int NST, int PMAX, bool BNB>
__global__ __launch_bounds__(WM* WN * 64) void conv3x3_patch_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NT = WM * WN * 64, RP = NT / 8;  // threads; LDS rows per load pass
  constexpr int BV = BN / RP;                    // weight-tile loads per thread per step
  constexpr int BSTAGE = BN * 128;
  static_assert(BV * RP == BN && NST >= 2 && NST <= 4, "config");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int S = p.splits;
  const int tile = bid / S, split = bid - tile * S;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int chunk = (tid & 7) ^ ((tid >> 4) & 7);  // source chunk of the lane-linear DMA image
  const int W2 = p.W + 2;

  char* ring = smem;
  char* patch = smem + NST * BSTAGE;
  const int pbytes = p.patch_rows * 128;

  // the block's input patch: padded rows [lbase, lbase + prows)
  const int mlast = min(m0 + BM, p.M) - 1;
  const int lbase = patch_lp(p, m0);
  const int prows = patch_lp(p, mlast) + 2 * W2 + 3 - lbase;
  const int passes = (prows + RP - 1) / RP;  // <= PMAX and passes * RP <= patch_rows (launcher)
  uint32_t poff[PMAX];  // byte offset of this thread's patch chunk, channel slab 0
  {
    const int HW2 = (p.H + 2) * W2;
#pragma unroll
    for (int v = 0; v < PMAX; ++v) {
      const int j = v * RP + (tid >> 3);
      uint32_t o = HCB_OOB;
      if (j < prows) {
        const int L = lbase + j;
        const int n = (int)fdiv((uint32_t)L, p.fd_hw2), rem = L - n * HW2;
        const int hh = (int)fdiv((uint32_t)rem, p.fd_w2), ww = rem - hh * W2;
        if (n < p.N && hh >= 1 && hh <= p.H && ww >= 1 && ww <= p.W)
          o = (uint32_t)((((n * p.H + hh - 1) * p.W + ww - 1) * p.ldx + chunk * 8) * 2);
      }
      poff[v] = o;
    }
  }
  // this lane's fragment rows in the patch (rows past M read a valid row; discarded)
  int prow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * TM + i * 16 + (lane & 15);
    prow[i] = patch_lp(p, m <= mlast ? m : mlast) - lbase;
  }
  uint32_t b_off[BV];
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const int j = n0 + (tid >> 3) + RP * v;
    b_off[v] = (j < p.Nout) ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
  }
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, p.w_bytes);

  // this split's channel slabs
  const int CS = p.C / 64;
  const int cs0 = split * CS / S, nslab = (split + 1) * CS / S - cs0;
  const int nk = nslab * 9;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  EpiPrefetch<WM, WN, TM, TN, BNB> pre;
  pre.load_shift(p, n0, wn, lane);
  const size_t param_off = patch_param_off<BM, BN, WM, NST>(p);
  if constexpr (BNB) stage_bnb_params<BN, NT>(p, n0, smem + param_off);  // published by the first barrier

  auto load_patch = [&](int sl) {  // the patch of local slab sl into buffer sl & 1
    char* pb = patch + (sl & 1) * pbytes;
    const uint32_t cb = (uint32_t)(cs0 + sl) * 128u;
#pragma unroll
    for (int v = 0; v < PMAX; ++v)
      if (v < passes) glds16(xr, pb + (wid * 8 + RP * v) * 128, poff[v] + cb);
  };
  // group g: the weight tile of step g, then (tap NST-1 of a slab with a successor) the next
  // slab's patch
  auto carries = [&](int g) { return g % 9 == NST - 1 && g / 9 + 1 < nslab; };
  auto issue = [&](int g) {
    const int sl = g / 9, t = g - sl * 9;
    char* sb = ring + (g % NST) * BSTAGE;
    const uint32_t kb = (uint32_t)(t * p.C + (cs0 + sl) * 64) * 2u;
#pragma unroll
    for (int v = 0; v < BV; ++v)
      glds16(wr, sb + (wid * 8 + RP * v) * 128, b_off[v] == HCB_OOB ? HCB_OOB : b_off[v] + kb);
    if (carries(g)) load_patch(sl + 1);
  };

  load_patch(0);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s);
  for (int k = 0; k < nk; ++k) {
    // group k has landed once only the loads issued after its weight tile are outstanding:
    // its own patch loads (if it carries the next patch) and the groups k+1 .. k+ahead
    const int ahead = min(NST - 2, nk - 1 - k);
    int cnt = carries(k) ? passes : 0;
    for (int a = 1; a <= ahead; ++a) cnt += BV + (carries(k + a) ? passes : 0);
    wait_vmcnt_rt(cnt);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + NST - 1 < nk) issue(k + NST - 1);
    const int sl = k / 9, t = k - sl * 9;
    const int r = t / 3;
    mfma_patch_step<WM, WN, TM, TN>(reinterpret_cast<const u32x4*>(patch + (sl & 1) * pbytes),
                                    reinterpret_cast<const u32x4*>(ring + (k % NST) * BSTAGE), prow,
                                    r * W2 + (t - 3 * r), acc, wn, lane);
  }
  __syncthreads();  // every wave is done reading before the epilogue reuses LDS
  if (S > 1 && !splitk_gather<MI, NI, NT>(p, acc, smem, tile, split, S, tid)) return;
  igemm_epilogue<WM, WN, TM, TN, BNB>(p, acc, smem, tm, m0, n0, wm, wn, lane, tid, pre, false, smem + param_off);
}

// ============================================================== launch
bool conv3x3_patch_eligible(const ConvParams& p) {
  return p.R == 3 && p.S == 3 && p.stride_h == 1 && p.stride_w == 1 && p.pad_h == 1 && p.pad_w == 1 &&
         p.dil_h == 1 && p.dil_w == 1 && p.idil_h == 1 && p.idil_w == 1 && p.P == p.H && p.Q == p.W &&
         p.C % 64 == 0 && p.Kpad == p.K && !p.remap && p.w_lo == nullptr && p.splits <= p.C / 64;
}

// upper bound of a block's padded input span (rows) over all its BM-pixel output tiles:
// BM - 1 steps, +2 per output-row wrap, +(2W + 4) per image wrap, plus the 3x3 window's reach
static int patch_span_bound(const ConvParams& p, int BM) {
  const int w = (BM - 1 + p.W - 1) / p.W + 1;
  const int im = (BM - 1 + p.H * p.W - 1) / (p.H * p.W) + 1;
  return BM - 1 + 2 * w + (2 * p.W + 4) * im + 2 * (p.W + 2) + 3;
}

template <typename K>
static void set_lds_max(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int WM, int WN, int TM, int TN, int NST, int PMAX>
static bool launch_patch(ConvParams p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN, NT = WM * WN * 64, RP = NT / 8;
  const int span = patch_span_bound(p, BM);
  const int passes = (span + RP - 1) / RP;
  if (passes > PMAX) return false;
  p.patch_rows = passes * RP;
  p.fd_hw = make_fastdiv((uint32_t)(p.H * p.W));
  p.fd_w = make_fastdiv((uint32_t)p.W);
  p.fd_hw2 = make_fastdiv((uint32_t)((p.H + 2) * (p.W + 2)));
  p.fd_w2 = make_fastdiv((uint32_t)(p.W + 2));
  const bool bnb = p.bnb_acc != nullptr;
  const size_t main_b = patch_main_lds<BM, BN, WM, NST>(p);
  const size_t epi_b = igemm_epilogue_lds(BM, BN, WM, igemm_stage16(p));
  size_t lds = main_b > epi_b ? main_b : epi_b;
  if (bnb) lds = patch_param_off<BM, BN, WM, NST>(p) + bnb_param_lds(BN);
  if (lds > 160 * 1024) return false;
  static bool once = false;
  if (!once) {
    set_lds_max(conv3x3_patch_kernel<WM, WN, TM, TN, NST, PMAX, false>);
    set_lds_max(conv3x3_patch_kernel<WM, WN, TM, TN, NST, PMAX, true>);
    once = true;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN) * p.splits;
  if (bnb)
    hipLaunchKernelGGL((conv3x3_patch_kernel<WM, WN, TM, TN, NST, PMAX, true>), dim3(tiles), dim3(NT), lds, st, p);
  else
    hipLaunchKernelGGL((conv3x3_patch_kernel<WM, WN, TM, TN, NST, PMAX, false>), dim3(tiles), dim3(NT), lds, st, p);
  return true;
}

// cfg 17: 128x128 (2x4 waves of 64x32), 18: 256x128 (4x2 of 64x64), 19: 256x64 (4x2 of 64x32),
// 20: 128x64 (2x2 of 64x32, 4 waves), 21: 128x128 with a 4-deep weight ring
bool launch_conv3x3_patch(const ConvParams& p, int cfg, hipStream_t st) {
  if (!conv3x3_patch_eligible(p)) return false;
  switch (cfg) {
    case 17: return launch_patch<2, 4, 64, 32, 3, 8>(p, st);
    case 18: return launch_patch<4, 2, 64, 64, 3, 8>(p, st);
    case 19: return launch_patch<4, 2, 64, 32, 3, 8>(p, st);
    case 20: return launch_patch<2, 2, 64, 32, 3, 16>(p, st);
    case 21: return launch_patch<2, 4, 64, 32, 4, 8>(p, st);
    default: return false;
  }
}

}  // namespace hcb
