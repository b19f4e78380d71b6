// fp32 convolutions on bf16 PLANES (the reference's precision, --compute_dtype fp32): every fp32
// GEMM operand is held in memory as three bf16 planes hi / mid / lo (x = hi + mid + lo exactly: 8 +
// 8 + 8 significant bits), written once by its PRODUCER (BN apply, BN backward, the plane-split
// kernel) where the split costs nothing -- those kernels are memory bound. The GEMMs then stage
// plain bf16 tiles: LDS-DMA (buffer_load ... lds) of 3 images per operand, no register staging, no
// VALU split, and six MFMA products per (A, B) fragment set (bf16x6: hi*hi + hi*mid + mid*hi +
// mid*mid + hi*lo + lo*hi, fp32 accumulation; the dropped mid*lo, lo*mid, lo*lo are ~2^-24).
//
// Roles (the reference's MKL-DNN fp32 Conv2D fwd / bwd-data / bwd-filter primitives, SURVEY.md
// §2.6, driven by /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81):
//   * conv_igemm_p3_kernel  forward and data-gradient implicit GEMMs (fp32 output, fused BN
//                           statistics, beta-accumulate, split-K via splitk_gather)
//   * conv_wgrad_p3_kernel  weight-gradient implicit GEMM (transposed fragment reads,
//                           ds_read_b64_tr_b16, split-K with fp32 atomics)
//
// Design for CDNA4: bf16x6 does 6 MFMAs per 3+3 fragment reads, twice the MFMA work per LDS byte
// of the bf16 GEMM, so these kernels can be MFMA bound -- the constraint is LDS CAPACITY (3 images
// per operand): a 128x64 block tile is 72 KB per k-step, so the ring is two stages (144 KB, one
// workgroup per CU). Each stage carries 6x the MFMA time of a bf16 k-step (1536 cycles per wave at
// 64x32 wave tiles), which covers the next stage's DMA latency, so double buffering is enough.
#include "conv_p3_fwd.h"

namespace hcb {

constexpr int N_P3_CFG = 18;
int p3_tile_m(int cfg) {
  static const int t[N_P3_CFG] = {128, 64, 128, 64, 64, 128, 64, 128, 128, 128, 256, 128, 64, 128, 128, 64, 64, 64};
  return (cfg >= 0 && cfg < N_P3_CFG) ? t[cfg] : 128;
}
int p3_slot_k(int cfg) { return (cfg >= 0 && cfg <= 6) ? 64 : 32; }
int p3_tile_n(int cfg) {
  static const int t[N_P3_CFG] = {64, 128, 64, 128, 64, 64, 128, 128, 128, 128, 128, 256, 128, 64, 64, 128, 64, 64};
  return (cfg >= 0 && cfg < N_P3_CFG) ? t[cfg] : 64;
}

void launch_conv_p3(const ConvParams& p, int cfg, hipStream_t st) {
  if (p.sk_grid > 0) {
    launch_conv_p3_sk(p, cfg, st);
    return;
  }
  if (p.bnb_acc != nullptr)
    launch_p3_cfg<true, false>(p, cfg, st);
  else
    launch_p3_cfg<false, false>(p, cfg, st);
}
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
// barrier per slot.
template <int WM, int WN, int TM, int TN, int NST, int BK, bool CBIG, int OCC = 1>
__global__ __launch_bounds__(WM* WN * 64, OCC* WM* WN / 4) void conv_wgrad_p3_kernel(WgradParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16, KS = BK / 32;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;        // 16-byte chunks per LDS row
  constexpr int ARPI = 64 / ACPR, BRPI = 64 / BCPR;  // LDS rows filled by one wave instruction
  constexpr int AI = BK / ARPI / NW, BI = BK / BRPI / NW;  // instructions per wave per plane and slot
  constexpr int LOADS = 3 * (AI + BI);
  constexpr int AIMG = BK * BM * 2, BIMG = BK * BN * 2;
  constexpr int STAGE = 3 * (AIMG + BIMG);
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

  auto issue = [&](int stage, int kl) {
    const int mb = mbeg + kl * BK;
    char* sA = smem + stage * STAGE;
    char* sB = sA + 3 * AIMG;
#pragma unroll
    for (int v = 0; v < AI; ++v) {
      const int m = mb + a_row[v];
      const uint32_t off = (a_col[v] < p.Nout && m < mend) ? (uint32_t)(m * p.ldy + a_col[v]) * 2u : HCB_OOB;
      char* d = sA + (wid * AI + v) * ARPI * BM * 2;
      glds16(dyr0, d, off);
      glds16(dyr1, d + AIMG, off);
      glds16(dyr2, d + 2 * AIMG, off);
    }
#pragma unroll
    for (int v = 0; v < BI; ++v) {
      const int m = mb + b_row[v];
      uint32_t off = HCB_OOB;
      if (b_ok[v] && m < mend) {
        const int n = (int)fdiv((uint32_t)m, p.fd_pq);
        const int rem = m - n * p.P * p.Q;
        const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
        const int qq = rem - pp * p.Q;
        const int h = pp * p.stride_h + b_dh[v], w = qq * p.stride_w + b_dw[v];
        if ((unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W)
          off = (uint32_t)(((n * p.H + h) * p.W + w) * p.ldx + b_c[v]) * 2u;
      }
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
    const char* Bb = Ab + 3 * AIMG;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int t = 0; t < 3; ++t) f.a[ks][t][i] = frag(Ab + t * AIMG, BM, ks * 32 + 8 * g, wm * TM + i * 16);
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t) f.b[ks][t][j] = frag(Bb + t * BIMG, BN, ks * 32 + 8 * g, wn * TN + j * 16);
    }
  };
  auto wait_ahead = [&](int ahead) {
    if (ahead >= 2)
      wait_vmcnt<(NST >= 3 ? 2 : 0) * LOADS>();
    else if (ahead == 1)
      wait_vmcnt<LOADS>();
    else
      wait_vmcnt<0>();
  };

  const int nk = (mend - mbeg + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < NST; ++s)
    if (s < nk) issue(s, s);
  constexpr int FREGS = (MI + NI) * 3 * 4 * KS, AREGS = MI * NI * 4;
  constexpr int RBUDGET = p3_regs_per_wave<OCC, WM * WN>() - 88 < 400 ? p3_regs_per_wave<OCC, WM * WN>() - 88 : 400;
  constexpr bool PIPE = 2 * FREGS + AREGS <= RBUDGET;
  if constexpr (PIPE) {
    Fr fr[2];
    if (nk > 0) {
      wait_ahead(min(NST - 1, nk - 1));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(0, fr[0]);
    }
    auto body = [&](int k, Fr& cur, Fr& nxt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot k are done
      if (k + 1 < nk) wait_ahead(min(NST - 2, nk - 2 - k));  // slot k+1 landed for this thread
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (k + NST < nk) issue(k % NST, k + NST);
      if (k + 1 < nk) read(k + 1, nxt);
      __builtin_amdgcn_sched_barrier(0);
      p3_mma<TM, TN, KS>(cur, acc);
    };
    for (int k = 0; k < nk; k += 2) {
      body(k, fr[0], fr[1]);
      if (k + 1 < nk) body(k + 1, fr[1], fr[0]);
    }
  } else {
    Fr fr;
    for (int k = 0; k < nk; ++k) {
      wait_ahead(min(NST - 1, nk - 1 - k));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(k, fr);
      if (k + NST < nk) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot are done
        __builtin_amdgcn_s_barrier();                        // ... and every other wave's
        asm volatile("" ::: "memory");
        issue(k % NST, k + NST);
      }
      p3_mma<TM, TN, KS>(fr, acc);
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
  const size_t lds_main = (size_t)NST * 3 * BK * (BM + BN) * 2;
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

// p3 wgrad cfg (block tile, waves x wave tile, slots x pixel rows):
//   0 128x64 (2x2 of 64x32, 2x64), 1 64x128 (2x2 of 32x64, 2x64), 2 64x64 (2x2 of 32x32, 3x64),
//   3 128x64 (4x2 of 32x32, 2x64), 4 64x128 (2x4 of 32x32, 2x64), 5 64x64 (2x2 of 32x32, 2x64),
//   6 128x128 (2x4 of 64x32, 3x32), 7 128x128 (4x2 of 32x64, 3x32), 8 256x128 (4x2 of 64x64, 2x32),
//   9 128x256 (2x4 of 64x64, 2x32), 10 128x128 (2x2 of 64x64, 3x32), 11 128x64 (2x2 of 64x32, 3x32),
//   two per CU: 12 128x64 (2x2 of 64x32, 2x32), 13 64x128 (2x2 of 32x64, 2x32), 14 64x64 (2x2 of 32x32, 3x32),
//   three per CU: 15 64x64 (2x2 of 32x32, 2x32)
constexpr int N_WP3_CFG = 16;
int wgrad_p3_tile_m(int cfg) {
  static const int t[N_WP3_CFG] = {128, 64, 64, 128, 64, 64, 128, 128, 256, 128, 128, 128, 128, 64, 64, 64};
  return (cfg >= 0 && cfg < N_WP3_CFG) ? t[cfg] : 64;
}
int wgrad_p3_tile_n(int cfg) {
  static const int t[N_WP3_CFG] = {64, 128, 64, 64, 128, 64, 128, 128, 128, 256, 128, 64, 64, 128, 64, 64};
  return (cfg >= 0 && cfg < N_WP3_CFG) ? t[cfg] : 64;
}

void launch_wgrad_p3(const WgradParams& p, int cfg, int splits, hipStream_t st) {
  switch (cfg) {
    case 0: wlaunch_p3<2, 2, 64, 32, 2, 64>(p, splits, st); break;
    case 1: wlaunch_p3<2, 2, 32, 64, 2, 64>(p, splits, st); break;
    case 3: wlaunch_p3<4, 2, 32, 32, 2, 64>(p, splits, st); break;
    case 4: wlaunch_p3<2, 4, 32, 32, 2, 64>(p, splits, st); break;
    case 5: wlaunch_p3<2, 2, 32, 32, 2, 64>(p, splits, st); break;
    case 6: wlaunch_p3<2, 4, 64, 32, 3, 32>(p, splits, st); break;
    case 7: wlaunch_p3<4, 2, 32, 64, 3, 32>(p, splits, st); break;
    case 8: wlaunch_p3<4, 2, 64, 64, 2, 32>(p, splits, st); break;
    case 9: wlaunch_p3<2, 4, 64, 64, 2, 32>(p, splits, st); break;
    case 10: wlaunch_p3<2, 2, 64, 64, 3, 32>(p, splits, st); break;
    case 11: wlaunch_p3<2, 2, 64, 32, 3, 32>(p, splits, st); break;
    case 12: wlaunch_p3<2, 2, 64, 32, 2, 32, 2>(p, splits, st); break;
    case 13: wlaunch_p3<2, 2, 32, 64, 2, 32, 2>(p, splits, st); break;
    case 14: wlaunch_p3<2, 2, 32, 32, 3, 32, 2>(p, splits, st); break;
    case 15: wlaunch_p3<2, 2, 32, 32, 2, 32, 3>(p, splits, st); break;
    default: wlaunch_p3<2, 2, 32, 32, 3, 64>(p, splits, st); break;
  }
}

// ============================================================== plane split / merge
// x fp32 [rows][ldx] (C channels used) -> three bf16 planes [3][rows][ldo] (plane stride `plane`
// elements): hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (round to nearest even;
// hi + mid + lo == x for every normal fp32 value)
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ x, int ldx, int C, int64_t n8,
                                                           uint16_t* __restrict__ out, int ldo, int64_t plane) {
  const int CV = C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / CV;
    const int cv = (int)(i - row * CV);
    const u32x4* src = reinterpret_cast<const u32x4*>(x + row * ldx + cv * 8);
    u32x4 hi, mid, lo;
    split3_8(src[0], src[1], hi, mid, lo);
    uint16_t* o = out + row * ldo + cv * 8;
    *reinterpret_cast<u32x4*>(o) = hi;
    *reinterpret_cast<u32x4*>(o + plane) = mid;
    *reinterpret_cast<u32x4*>(o + 2 * plane) = lo;
  }
}

__global__ __launch_bounds__(256) void merge_planes_kernel(const uint16_t* __restrict__ in, int ldi, int64_t plane,
                                                           int C, int64_t n8, float* __restrict__ y, int ldy) {
  const int CV = C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / CV;
    const int cv = (int)(i - row * CV);
    const uint16_t* s = in + row * ldi + cv * 8;
    float h[8], m[8], l[8];
    unpack_bf16x8(*reinterpret_cast<const u32x4*>(s), h);
    unpack_bf16x8(*reinterpret_cast<const u32x4*>(s + plane), m);
    unpack_bf16x8(*reinterpret_cast<const u32x4*>(s + 2 * plane), l);
    float* o = y + row * ldy + cv * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = h[e] + (m[e] + l[e]);
  }
}

// global average pool on planes (the ResNet head on the fp32 path): x planes [N][HW][C] -> the
// pooled features as planes [N][C] (the classifier GEMM's operand); fp32 sums of the exact values
__global__ __launch_bounds__(256) void gap_fwd_p3_kernel(const uint16_t* __restrict__ x, int64_t xps,
                                                         uint16_t* __restrict__ y, int64_t yps, int N, int HW, int C) {
  const int CV = C >> 3;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * CV) return;
  const int n = idx / CV, cv = idx % CV;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < HW; ++i) {
    const uint16_t* s = x + ((size_t)n * HW + i) * C + cv * 8;
    float f[8];
    merge_p3(*reinterpret_cast<const u32x4*>(s), *reinterpret_cast<const u32x4*>(s + xps),
             *reinterpret_cast<const u32x4*>(s + 2 * xps), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += f[e];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] *= inv;
  store_p3(y + (size_t)n * C + cv * 8, yps, acc);
}

void launch_gap_fwd_p3(const uint16_t* x, int64_t xps, uint16_t* y, int64_t yps, int N, int HW, int C, hipStream_t st) {
  const int total = N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_p3_kernel, dim3((total + 255) / 256), dim3(256), 0, st, x, xps, y, yps, N, HW, C);
}

static int p3_grid(int64_t n8) {
  int64_t b = (n8 + 255) / 256;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

void launch_split_planes(const float* x, int ldx, int64_t rows, int C, uint16_t* out, int ldo, int64_t plane,
                         hipStream_t st) {
  const int64_t n8 = rows * (C / 8);
  hipLaunchKernelGGL(split_planes_kernel, dim3(p3_grid(n8)), dim3(256), 0, st, x, ldx, C, n8, out, ldo, plane);
}

void launch_merge_planes(const uint16_t* in, int ldi, int64_t plane, int64_t rows, int C, float* y, int ldy,
                         hipStream_t st) {
  const int64_t n8 = rows * (C / 8);
  hipLaunchKernelGGL(merge_planes_kernel, dim3(p3_grid(n8)), dim3(256), 0, st, in, ldi, plane, C, n8, y, ldy);
}

}  // namespace hcb
