// Persistent forward / data-gradient plane GEMM (bf16x6, fp32 output) for SHORT-K problems: the
// stage-1 1x1 convs (K = 64 / 256: two to eight 32-deep k-steps per tile), the space-to-depth stem
// (K = 256) and the other layers whose tiles are too short for the per-workgroup prologue (first
// DMA round trip) and epilogue (LDS staging, barriers, stores) to hide behind their own MFMAs.
//
// conv_igemm_p3_kernel runs one output tile per workgroup: every tile pays a DMA latency before
// its first MFMA and drains its ring before its epilogue, and with 2-8 k-steps that is most of the
// tile's life (stage-1 64->256 forward: 103 us where its 282 MB of traffic needs ~56 us). Here a
// workgroup owns tiles first, first + grid, ... (grid = resident workgroups) and the LDS-DMA ring
// never drains: the k-step stream runs across tile boundaries, so the next tile's first slots are
// in flight while the current tile's last MFMAs and its epilogue run. The epilogue works from the
// accumulator registers -- no LDS staging, no barrier: BN statistics by two xor-shuffles and one
// buffer atomic per column and wave, the output by one dword buffer store per accumulator element
// (16 lanes write 64 contiguous bytes; the two 16-column halves of a 128-byte line land together
// in L2) -- so the ring (NST slots) plus a BN-shift table is the kernel's whole LDS.
//
// vmcnt accounting: every slot issue is LOADS LDS-DMA pieces (dummy pieces past the last tile,
// out of range), and every epilogue is EXACTLY EOPS vector-memory instructions per thread (masked
// elements store / add to an out-of-range offset instead of being branched around), so "slot
// g+1 has landed" is a compile-time count: NST-2 later slot issues, plus EOPS when the previous
// tile's epilogue was issued after slot g+1's DMA (the first NST-1 steps of a tile).
//
// Not served (the host falls back to the twin cfg of conv_igemm_p3_kernel): the fused
// BN-backward epilogue, split-K, beta-accumulate, bias, the strided-output remap and the
// input-dilated (strided data-gradient) loader.
// The reference's role: the MKL-DNN fp32 Conv2D forward primitive, driven by
// /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:62-81.
#pragma once
#include <cstdlib>

#include "conv_p3_fwd.h"
#include "conv_p3_wgrad.h"

namespace hcb {

__device__ __forceinline__ void buf_store_f32(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
__device__ __forceinline__ void buf_atomic_add_f32(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, r, off, 0, 0);
}

// LDS of the persistent kernel: the ring and the BN-statistic shift of every output column
template <int BM, int BN, int KW, int NST>
constexpr size_t p3p_ring_bytes() {
  return (size_t)NST * p3_stage_bytes<BM, BN, KW>();
}

// STATS: BN statistics into p.stats_R replicas, replica = the wave's 64-row block (mod R). TM >= 32:
// a replica slot receives at most two adds per tile (the two 32-row waves of a 64-row block), and
// two fp32 adds commute exactly, so the deterministic mode's one-replica-per-64-rows statistics stay
// bitwise reproducible.
//
// SK (stream-K, cfg 23-27): instead of whole tiles first, first + grid, ... every workgroup owns a
// CONTIGUOUS share [x0, x0 + nsteps) of all ntiles x nk (tile, k-step) iterations, equal to within
// one k-step, so the launch has no wave-quantization tail (196 tiles of 128 x 128 on 256 CUs leave
// 60 CUs idle for the whole launch; here every CU runs ~0.77 tile). The ring runs across the share's
// tile boundaries as in the whole-tile form (no per-share ramp: round 4's stream-K paid one per
// share, profiles/r4v_streamk_probe.txt). A tile split between workgroups (its shares: the workgroups
// of its first .. last iteration, at most p.splits of them) meets through the split-K hand-off
// (splitk_gather's protocol: slab in p.ws, agent-scope release + ticket in p.cnt[tile]; the last
// arriver acquires, sums every share's slab in share order -- run-to-run deterministic -- and runs
// the epilogue). Only a share's first and last segments can be split tiles, so a workgroup pays at
// most two hand-offs, and the spin-free protocol cannot deadlock whatever the residency.
//
// BNB (a data gradient whose output is a BN layer's dy, conv_p3_fwd.h's fused BN-backward epilogue
// from the registers): per tile, z (fp32), the ReLU-mask source (mode 1: the bf16 hi plane of y) and
// the beta-accumulate source (fp32) of the lane's accumulator elements are loaded in two chunks of
// wave rows (one memory round trip each), g = (acc [+ beta]) gated, stored fp32, and sum(g) /
// sum(g * xhat) reduced per column by shuffles into one buffer atomic per column and wave (replica =
// the wave's 64-row block, as the statistics) -- EOPS vector-memory instructions after the loads.
//
// BRES (B resident, cfg 31-36): the workgroup's whole weight slice (its N tile's every k-step: three
// plane images, nk * 3 * BN * 64 B) is DMA'd into LDS once, and the ring streams A only. The host
// sizes the grid as a multiple of the N-tile count, so first, first + grid, ... all lie in the N tile
// first % tiles_n. For the 1x1 GEMMs with K <= 256 the weight tile is as large as the activation
// tile or larger (stage 1, 64 -> 256: BN x K = 256 x 64 against BM x K = 64 x 64), so re-staging it
// for every tile doubled-to-quintupled the L2 -> LDS operand traffic that bounds these launches.
template <int WM, int WN, int TM, int TN, int KW, int NST, bool CBIG, bool STATS, int OCC, bool SK = false,
          bool BNB = false, bool BRES = false>
__global__ __launch_bounds__(WM* WN * 64, OCC* WM* WN / 4) void conv_p3_persist_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NT = WM * WN * 64, CPR = KW / 8, RB = KW * 2;
  constexpr int RP = NT / CPR;
  constexpr int AV = BM / RP, BV = BN / RP;
  static_assert(!(BRES && (SK || BNB)), "B-resident: the whole-tile forward form");
  constexpr int LOADS = NPL * (AV + (BRES ? 0 : BV));
  constexpr int AIMG = BM * RB, BIMG = BN * RB;
  constexpr int STAGE = BRES ? NPL * AIMG : (int)p3_stage_bytes<BM, BN, KW>();
  // epilogue vector-memory instructions; EDRAIN (64 x 64 wave tiles: more than the vmcnt field can
  // count beside the ring): the epilogue drains itself instead and the ring's waits count 0 for it
  static_assert(!(STATS && BNB), "a data gradient has no forward statistics");
  constexpr int EOPS_N = MI * NI * 4 + (STATS || BNB ? 2 * NI : 0);
  constexpr bool EDRAIN = LOADS * (NST - 1) + EOPS_N > 63;
  constexpr int EOPS = EDRAIN ? 0 : EOPS_N;
  static_assert(TM >= 32, "at most two adds per statistics slot and tile (deterministic mode)");
  static_assert(AV * RP == BM && (BRES || BV * RP == BN), "tile rows must be a multiple of the load pass");
  static_assert(LOADS * (NST - 1) + EOPS <= 63 && NST >= 2 && NST <= 4, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // BRES: the resident weight images after the A ring, then the shift table
  char* bres = smem + (size_t)NST * STAGE;
  const size_t bres_bytes = BRES ? (size_t)(p.Kpad / KW) * NPL * BIMG : 0;
  float* ktab = reinterpret_cast<float*>(smem + (size_t)NST * STAGE + bres_bytes);
  // SK: the last-arriver broadcast word, after the shift table
  int* skflag = reinterpret_cast<int*>(smem + (size_t)NST * STAGE + bres_bytes + (STATS ? (size_t)p.Nout * 4 : 0));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
  const int wm = wid / WN, wn = wid % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int ntiles = ((p.M + BM - 1) / BM) * tiles_n;
  const int grid = gridDim.x;
  const int first = xcd_remap(blockIdx.x, grid);  // concurrent neighbours (same M rows) share an XCD
  const int nk = p.Kpad / KW;
  // the work: SK -- iterations [x0, x0 + nsteps) of the tile-major (tile, k-step) space; otherwise
  // `mine` whole tiles first, first + grid, ...
  int mine = 0, x0 = 0, nsteps = 0;
  if constexpr (SK) {  // 32-bit: the host checks ntiles * nk * grid < 2^32
    const uint32_t T = (uint32_t)ntiles * (uint32_t)nk;
    x0 = (int)((uint32_t)first * T / (uint32_t)grid);
    nsteps = (int)((uint32_t)(first + 1) * T / (uint32_t)grid) - x0;
    if (nsteps <= 0) return;  // uniform (the host sizes grid <= ntiles * nk)
  } else {
    if (first >= ntiles) return;  // uniform (the host sizes grid <= ntiles)
    mine = (ntiles - 1 - first) / grid + 1;
    nsteps = mine * nk;
  }
  const int chunk = (tid % CPR) ^ p3_swz<KW>(tid / CPR);

  const char* xb = reinterpret_cast<const char*>(p.x);
  const __amdgpu_buffer_rsrc_t xr0 = make_rsrc(xb, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr1 = make_rsrc(xb + p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr2 = make_rsrc(xb + 2 * (size_t)p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr0 = make_rsrc(p.w, p.w_bytes);
  const __amdgpu_buffer_rsrc_t wr1 = make_rsrc(p.w_lo, p.w_bytes);
  const __amdgpu_buffer_rsrc_t wr2 = make_rsrc(p.w_lo2, p.w_bytes);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, (uint32_t)((size_t)p.M * p.ldy * 4));
  const __amdgpu_buffer_rsrc_t sr = BNB ? make_rsrc(p.bnb_acc, (uint32_t)((size_t)p.bnb_R * 2 * p.Nout * 4))
                                       : make_rsrc(p.stats, STATS ? (uint32_t)((size_t)p.stats_R * 2 * p.Nout * 4) : 0u);
  // BNB operands: z and the beta source fp32 (row strides bnb_ld / ldy), y's hi plane bf16 (bnb_ld)
  const __amdgpu_buffer_rsrc_t zr = make_rsrc(BNB ? p.bnb_z : p.y, BNB ? (uint32_t)((size_t)p.M * p.bnb_ld * 4) : 0u);
  const __amdgpu_buffer_rsrc_t br = make_rsrc(BNB && p.beta ? p.yres : p.y, BNB && p.beta ? (uint32_t)((size_t)p.M * p.ldy * 4) : 0u);
  const __amdgpu_buffer_rsrc_t mr = make_rsrc(BNB && p.bnb_mode == 1 ? p.bnb_y : p.y,
                                              BNB && p.bnb_mode == 1 ? (uint32_t)((size_t)p.M * p.bnb_ld * 2) : 0u);

  if constexpr (STATS) {  // published by the first barrier; older than every DMA (vmcnt order)
    for (int c = tid; c < p.Nout; c += NT) ktab[c] = p.stats_shift != nullptr ? p.stats_shift[c] : 0.f;
  }

  // ---- issue cursor: the (local tile, k-step) whose slot is issued next, NST steps ahead of the
  // MFMAs; its loader state follows it across tile boundaries
  ALoader<AV, CBIG, false, RP, 2, KW> al;
  uint32_t b_off[BV > 0 ? BV : 1];
  int ci = 0, ck = 0;  // the next issue: local tile (whole-tile form) / local step (SK), and k-step
  auto cursor_at = [&](int t, int k0) {
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    al.init(p, tm * BM, tid, chunk);
    if (k0 > 0) al.seek(p, k0);
#pragma unroll
    for (int v = 0; v < (BRES ? 0 : BV); ++v) {  // (BRES stages its weights itself)
      const int j = tn * BN + tid / CPR + RP * v;
      b_off[v] = (j < p.Nout) ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
    }
  };
  auto cursor_tile = [&](int i) { cursor_at(first + i * grid, 0); };
  if constexpr (SK) {
    ck = x0 % nk;
    cursor_at(x0 / nk, ck);
  } else {
    cursor_tile(0);
  }
  constexpr int WROWS = 64 / CPR;
  // branch-free: past the last tile every piece is out of range (lands zeros in a slot nobody reads)
  auto issue = [&](int stage) {
    const bool live = SK ? ci < nsteps : ci < mine;
    uint32_t off[AV];
    al.offsets(p, ck, chunk, off);
    char* sa = smem + stage * STAGE + wid * WROWS * RB;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const uint32_t o = live ? off[v] : HCB_OOB;
      glds16(xr0, sa + RP * v * RB, o);
      glds16(xr1, sa + AIMG + RP * v * RB, o);
      glds16(xr2, sa + 2 * AIMG + RP * v * RB, o);
    }
    if constexpr (!BRES) {
      char* sb = smem + stage * STAGE + NPL * AIMG + wid * WROWS * RB;
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        const uint32_t o = (b_off[v] == HCB_OOB || !live) ? HCB_OOB : b_off[v] + (uint32_t)ck * (uint32_t)RB;
        glds16(wr0, sb + RP * v * RB, o);
        glds16(wr1, sb + BIMG + RP * v * RB, o);
        glds16(wr2, sb + 2 * BIMG + RP * v * RB, o);
      }
    }
  };
  auto advance = [&]() {
    if constexpr (SK) {
      ++ci;
      if (++ck == nk) {
        ck = 0;
        if (ci < nsteps) cursor_at((x0 + ci) / nk, 0);
      }
    } else {
      if (++ck == nk) {
        ck = 0;
        if (++ci < mine) cursor_tile(ci);
      }
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- register epilogue of tile t: exactly EOPS vector-memory instructions per thread
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    const int rbase = tm * BM + wm * TM;           // the wave's first row
    const int cbase = tn * BN + wn * TN + frow;    // the lane's column in fragment j = 0
    if constexpr (BNB) {
      float mu[NI], is[NI], sc[NI], sh[NI], s1[NI], s2[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = cbase + j * 16;
        const bool cok = col < p.Nout;
        mu[j] = cok ? p.bnb_mean[col] : 0.f;
        is[j] = cok ? p.bnb_invstd[col] : 0.f;
        sc[j] = (cok ? p.bnb_gamma[col] : 0.f) * is[j];
        sh[j] = (cok ? p.bnb_beta[col] : 0.f) - mu[j] * sc[j];
        s1[j] = 0.f;
        s2[j] = 0.f;
      }
      const int mode = p.bnb_mode;
      const bool beta = p.beta != 0;
      constexpr int HC = MI > 1 ? MI / 2 : 1;  // wave-row fragments per chunk
#pragma unroll
      for (int c0 = 0; c0 < MI; c0 += HC) {
        float zf[HC][4][NI], rf[HC][4][NI];
        uint32_t yb[HC][4][NI];
#pragma unroll
        for (int ii = 0; ii < HC; ++ii)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = rbase + (c0 + ii) * 16 + fq * 4 + e;
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              const int col = cbase + j * 16;
              const bool ok = (row < p.M) & (col < p.Nout);
              zf[ii][e][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                  zr, ok ? (uint32_t)(row * p.bnb_ld + col) * 4u : HCB_OOB, 0, 0));
              rf[ii][e][j] = beta ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                        br, ok ? (uint32_t)(row * p.ldy + col) * 4u : HCB_OOB, 0, 0))
                                  : 0.f;
              yb[ii][e][j] = mode == 1 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(
                                             mr, ok ? (uint32_t)(row * p.bnb_ld + col) * 2u : HCB_OOB, 0, 0)
                                       : 0u;
            }
          }
#pragma unroll
        for (int ii = 0; ii < HC; ++ii)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = rbase + (c0 + ii) * 16 + fq * 4 + e;
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              const int col = cbase + j * 16;
              const bool ok = (row < p.M) & (col < p.Nout);
              const float z = zf[ii][e][j];
              float g = acc[c0 + ii][j][e] + rf[ii][e][j];
              if (mode == 1)
                g = __uint_as_float(yb[ii][e][j] << 16) > 0.f ? g : 0.f;  // the hi plane: > 0 exactly when y > 0
              else if (mode == 2)
                g = (z * sc[j] + sh[j]) > 0.f ? g : 0.f;
              g = ok ? g : 0.f;
              s1[j] += g;
              s2[j] += g * ((z - mu[j]) * is[j]);
              buf_store_f32(yr, ok ? (uint32_t)(row * p.ldy + col) * 4u : HCB_OOB, g);
            }
          }
      }
      const uint32_t rep = (uint32_t)((rbase >> 6) % p.bnb_R) * 2u * (uint32_t)p.Nout;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        float a = s1[j], b = s2[j];
        a += __shfl_xor(a, 16, 64);
        b += __shfl_xor(b, 16, 64);
        a += __shfl_xor(a, 32, 64);
        b += __shfl_xor(b, 32, 64);
        const int col = cbase + j * 16;
        const bool own = (fq == 0) & (col < p.Nout);
        buf_atomic_add_f32(sr, own ? (rep + (uint32_t)col) * 4u : HCB_OOB, a);
        buf_atomic_add_f32(sr, own ? (rep + (uint32_t)(p.Nout + col)) * 4u : HCB_OOB, b);
      }
      if constexpr (EDRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    if constexpr (STATS) {
      const int wrows = p.M - rbase;
      const uint32_t rep = (uint32_t)((rbase >> 6) % p.stats_R) * 2u * (uint32_t)p.Nout;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = cbase + j * 16;
        const bool cok = col < p.Nout;
        const float kc = cok ? ktab[col] : 0.f;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int ii = 0; ii < MI; ++ii)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = ii * 16 + fq * 4 + e < wrows ? acc[ii][j][e] - kc : 0.f;
            s1 += v;
            s2 += v * v;
          }
        s1 += __shfl_xor(s1, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        const bool own = (fq == 0) & cok;
        const uint32_t o1 = own ? (rep + (uint32_t)col) * 4u : HCB_OOB;
        const uint32_t o2 = own ? (rep + (uint32_t)(p.Nout + col)) * 4u : HCB_OOB;
        buf_atomic_add_f32(sr, o1, s1);
        buf_atomic_add_f32(sr, o2, s2);
      }
    }
    const bool relu = p.relu != 0;
#pragma unroll
    for (int ii = 0; ii < MI; ++ii)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + ii * 16 + fq * 4 + e;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int col = cbase + j * 16;
          const bool ok = (row < p.M) & (col < p.Nout);
          const uint32_t o = ok ? (uint32_t)(row * p.ldy + col) * 4u : HCB_OOB;
          const float v = acc[ii][j][e];
          buf_store_f32(yr, o, relu ? fmaxf(v, 0.f) : v);
        }
      }
    if constexpr (EDRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int ii = 0; ii < MI; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // ---- SK: a split tile's segment ends here. Park the partial, take a ticket; the last of the
  // tile's S shares sums every slab in share order and runs the epilogue. Drains this thread's
  // vector memory (the ring's in-flight slots included: the later counted waits only get stricter)
  auto partial = [&](int t) __attribute__((always_inline)) {
    constexpr int FR = MI * NI;
    if (p.cnt == nullptr) {  // timing probe only (HCB_SK_PROBE=1): no hand-off, the split tiles' output is wrong
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    const uint32_t T = (uint32_t)ntiles * (uint32_t)nk;
    // the share holding iteration x: the largest w with w * T / grid <= x
    auto owner = [&](uint32_t x) { return (int)(((x + 1) * (uint32_t)grid - 1) / T); };
    const int w0 = owner((uint32_t)(t * nk)), S = owner((uint32_t)((t + 1) * nk - 1)) - w0 + 1;
    f32x4* slab = reinterpret_cast<f32x4*>(p.ws) + (size_t)t * p.splits * FR * NT;
    // the partial leaves by sc1 (write-through) stores, drained by every storing wave before the
    // ticket: no agent-scope release, whose L2 write-back of EVERY dirty line of the XCD (this
    // launch's whole output stream) cost ~6x the kernel's time (MI355X guide, publish-large); the
    // last arriver still acquires before reading the slabs
    const __amdgpu_buffer_rsrc_t wsr = make_rsrc(p.ws, (uint32_t)(p.ws_floats * 4 < 0x7fffffff ? p.ws_floats * 4 : 0x7fffffff));
    const uint32_t sbase = (uint32_t)(((size_t)t * p.splits + (first - w0)) * FR * NT + tid) * 16u;
#pragma unroll
    for (int ii = 0; ii < MI; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const f32x4 a = acc[ii][j];
        const u32x4 v = {__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3])};
        __builtin_amdgcn_raw_buffer_store_b128(v, wsr, sbase + (uint32_t)((ii * NI + j) * NT) * 16u, 0, 16 /* sc1 */);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned got = __hip_atomic_fetch_add(p.cnt + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = got == (unsigned)(S - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(p.cnt + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      *skflag = last;
    }
    __syncthreads();
    if (*skflag != 0) {
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[ii][j] = slab[(size_t)(ii * NI + j) * NT + tid];
      for (int sh = 1; sh < S; ++sh) {
#pragma unroll
        for (int ii = 0; ii < MI; ++ii)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[ii][j] += slab[((size_t)sh * FR + ii * NI + j) * NT + tid];
      }
      epilogue(t);
    } else {
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  auto read = [&](int g, P3Frags<TM, TN, KW / 32>& f) {
    const char* sb = smem + (g % NST) * STAGE;
    const char* bb = BRES ? bres + (size_t)(g % nk) * NPL * BIMG : sb + NPL * AIMG;  // BRES: step g's k-step
    p3_read<WM, WN, TM, TN, KW>(reinterpret_cast<const u32x4*>(sb), reinterpret_cast<const u32x4*>(bb), f, wm, wn, lane);
  };

  if constexpr (BRES) {  // every k-step's weight images of this workgroup's N tile, once
    const int n0 = (first % tiles_n) * BN;
    // rows rb .. rb + WROWS - 1 per wave instruction (wave-uniform; a wave past BN issues nothing):
    // the lane-linear images of issue()'s B part, row r's swizzle a function of tid as there
    for (int rb = wid * WROWS; rb < BN; rb += RP) {
      const int j = n0 + rb + lane / CPR;
      const uint32_t bo = j < p.Nout ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
      for (int kt = 0; kt < nk; ++kt) {
        char* sb = bres + (size_t)kt * NPL * BIMG + rb * RB;
        const uint32_t o = bo == HCB_OOB ? HCB_OOB : bo + (uint32_t)kt * (uint32_t)RB;
        glds16(wr0, sb, o);
        glds16(wr1, sb + BIMG, o);
        glds16(wr2, sb + 2 * BIMG, o);
      }
    }
    // landed before the ring starts (the ring's counted waits count ring pieces only); published to
    // the other waves by the first barrier below
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int s = 0; s < NST; ++s) {
    issue(s);
    advance();
  }
  constexpr int FREGS = (MI + NI) * NPL * 4 * (KW / 32), AREGS = MI * NI * 4;
  constexpr int RBUDGET = p3_regs_per_wave<OCC, WM * WN>() - 64 < 400 ? p3_regs_per_wave<OCC, WM * WN>() - 64 : 400;
  constexpr bool PIPE = 2 * FREGS + AREGS <= RBUDGET;
  constexpr int NMF = (KW / 32) * MI * NI * 6, NRD = (KW / 32) * (MI + NI) * NPL;
  int i = 0, k = 0;  // the compute side's local tile (SK: segment) and k-step
  // SK: the first segment starts at k-step x0 % nk (a later one at 0); k counts the steps since the
  // last segment end once one has ended (i > 0)
  if constexpr (SK) k = x0 % nk;
  // after the MFMAs of step g: the tile's epilogue once its last k-step is in (SK: the segment's
  // epilogue or hand-off at a tile end or the share's end)
  auto post = [&](int g) __attribute__((always_inline)) {
    if constexpr (SK) {
      const bool tile_end = ++k == nk;
      if (tile_end || g + 1 == nsteps) {
        const int t = (x0 + g) / nk;
        if (tile_end && (i > 0 || x0 % nk == 0))  // the segment ran the whole tile
          epilogue(t);
        else
          partial(t);
        ++i;
        k = 0;
      }
    } else {
      if (++k == nk) {
        epilogue(first + i * grid);
        k = 0;
        ++i;
      }
    }
  };
  // "an epilogue's EOPS instructions were issued after the awaited slot's DMA": the first steps after
  // a segment end (after an SK hand-off every older instruction has drained: any count is safe)
  auto after_epi = [&](int lim) { return i > 0 && k <= lim; };
  if constexpr (PIPE) {
    P3Frags<TM, TN, KW / 32> fr[2];
    wait_vmcnt<(NST - 1) * LOADS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, fr[0]);
    auto body = [&](int g, P3Frags<TM, TN, KW / 32>& cur, P3Frags<TM, TN, KW / 32>& nxt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot g are done
      // slot g+1 has landed for this thread
      if (after_epi(NST - 2))
        wait_vmcnt<(NST - 2) * LOADS + EOPS>();
      else
        wait_vmcnt<(NST - 2) * LOADS>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(g % NST);
      read(g + 1, nxt);
      p3_mma<TM, TN, KW / 32>(cur, acc);
      ilv_schedule<NMF, LOADS, NRD>();
      advance();
      post(g);
    };
    for (int g = 0; g < nsteps; g += 2) {
      body(g, fr[0], fr[1]);
      if (g + 1 < nsteps) body(g + 1, fr[1], fr[0]);
    }
  } else {
    P3Frags<TM, TN, KW / 32> fr;
    for (int g = 0; g < nsteps; ++g) {
      // slot g has landed: NST-1 later slot issues, plus the previous epilogue when it came after
      if (after_epi(NST - 1))
        wait_vmcnt<(NST - 1) * LOADS + EOPS>();
      else
        wait_vmcnt<(NST - 1) * LOADS>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(g, fr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(g % NST);
      p3_mma<TM, TN, KW / 32>(fr, acc);
      ilv_schedule<NMF, LOADS, 0>();
      advance();
      post(g);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy pieces have landed before the LDS is freed
}

// kernels.h set_p3p_bnb
inline int& p3p_bnb_level() {
  static int v = [] {
    const char* e = std::getenv("HCB_P3P_BNB");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  return v;
}

// cfg 18-22 (persistent twins of cfg 15, 14, 16, 17, 7): false when the problem needs an epilogue
// feature this kernel does not have (the caller then launches the twin). A fused BN-backward data
// gradient (bnb_acc) runs the BNB instantiation.
template <int WM, int WN, int TM, int TN, int KW, int NST, int OCC>
static bool launch_p3p(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  const bool stats = p.stats != nullptr;
  const int nk = p.Kpad / KW;
  const size_t ring = p3p_ring_bytes<BM, BN, KW, NST>();
  const size_t lds = ring + (stats ? (size_t)p.Nout * 4 : 0);
  const bool bnb = p.bnb_acc != nullptr;
  // the mode-1 mask is a 2-byte load per accumulator element (the hi plane of y): measured slower
  // than the twin's vector prefetch, so only p3p_bnb_level() 2 runs it here
  if ((bnb && (p3p_bnb_level() == 0 || (p.bnb_mode == 1 && p3p_bnb_level() < 2))) || p.remap || p.idil_h > 1 || p.idil_w > 1 || p.splits != 1 || (p.beta && !bnb) ||
      p.bias != nullptr || !p.out_f32 || (bnb && (stats || p.bnb_R <= 0 || p.bnb_mode < 0 || p.bnb_mode > 2)) ||
      (stats && p.stats_R <= 0) || nk < NST - 1 || p.Kpad % KW != 0 || lds > 160 * 1024 ||
      (size_t)p.M * p.ldy * 4 >= (1ull << 31) || (bnb && (size_t)p.M * p.bnb_ld * 4 >= (1ull << 31)))
    return false;
  const bool cbig = (p.C % KW) == 0;
  static bool once = false;
  if (!once) {
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, OCC, false, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, OCC, false, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, true, OCC>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, OCC>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, true, OCC>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, OCC>);
    once = true;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ntiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN);
  const int per_cu = (int)((160 * 1024) / lds) < OCC ? (int)((160 * 1024) / lds) : OCC;
  const int slots = cus * (per_cu > 0 ? per_cu : 1);
  const int grid = ntiles < slots ? ntiles : slots;
  const dim3 b(WM * WN * 64);
  if (bnb && cbig)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, OCC, false, true>), dim3(grid), b,
                       lds, st, p);
  else if (bnb)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, OCC, false, true>), dim3(grid),
                       b, lds, st, p);
  else if (cbig && stats)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, true, OCC>), dim3(grid), b, lds, st, p);
  else if (cbig)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, OCC>), dim3(grid), b, lds, st, p);
  else if (stats)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, true, OCC>), dim3(grid), b, lds, st, p);
  else
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, OCC>), dim3(grid), b, lds, st,
                       p);
  return true;
}

// cfg 31-34: the B-resident form (BRES above). False when the problem does not fit it (more than one
// N tile, the weights + ring over the LDS, an epilogue feature the persistent kernel lacks): the
// caller then runs the whole-tile persistent cfg.
template <int WM, int WN, int TM, int TN, int KW, int NST>
static bool launch_p3bres(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN, NPLc = NPL;
  const bool stats = p.stats != nullptr;
  const int nk = p.Kpad / KW;
  const size_t lds = (size_t)NST * NPLc * BM * KW * 2 + (size_t)nk * NPLc * BN * KW * 2 + (stats ? (size_t)p.Nout * 4 : 0);
  if (p.bnb_acc != nullptr || p.remap || p.idil_h > 1 || p.idil_w > 1 || p.splits != 1 || p.beta ||
      p.bias != nullptr || !p.out_f32 || (stats && p.stats_R <= 0) || nk < NST - 1 || p.Kpad % KW != 0 ||
      lds > 160 * 1024 || (size_t)p.M * p.ldy * 4 >= (1ull << 31))
    return false;
  const bool cbig = (p.C % KW) == 0;
  static bool once = false;
  if (!once) {
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, true, 1, false, false, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, 1, false, false, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, true, 1, false, false, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, 1, false, false, true>);
    once = true;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int ntiles = ((p.M + BM - 1) / BM) * tiles_n;
  const int per_cu = (int)((160 * 1024) / lds) < 1 ? 1 : (int)((160 * 1024) / lds);
  const int slots = cus * per_cu;
  // a multiple of the N-tile count: each workgroup's tiles share one N tile (its resident slice)
  const int grid = ((ntiles < slots ? ntiles : slots) / tiles_n) * tiles_n;
  if (grid <= 0) return false;
  const dim3 b(WM * WN * 64);
  if (cbig && stats)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, true, 1, false, false, true>), dim3(grid),
                       b, lds, st, p);
  else if (cbig)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, 1, false, false, true>), dim3(grid),
                       b, lds, st, p);
  else if (stats)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, true, 1, false, false, true>), dim3(grid),
                       b, lds, st, p);
  else
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, 1, false, false, true>), dim3(grid),
                       b, lds, st, p);
  return true;
}

// cfg 23-27: the stream-K form of cfg 18-22 (same tiles and ring). False when the problem needs an
// epilogue feature the persistent kernel does not have, or the split-K workspace cannot hold every
// tile's shares (the caller then tries the whole-tile persistent cfg, then the twin).
template <int WM, int WN, int TM, int TN, int KW, int NST, int OCC>
static bool launch_p3sk(const ConvParams& p0, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  ConvParams p = p0;
  const bool stats = p.stats != nullptr;
  const int nk = p.Kpad / KW;
  const size_t ring = p3p_ring_bytes<BM, BN, KW, NST>();
  const size_t lds = ring + (stats ? (size_t)p.Nout * 4 : 0) + 16;  // + the last-arriver word
  if (p.bnb_acc != nullptr || p.remap || p.idil_h > 1 || p.idil_w > 1 || p.splits != 1 || p.beta ||
      p.bias != nullptr || !p.out_f32 || p.ws == nullptr || p.cnt == nullptr ||
      (stats && p.stats_R <= 0) || nk < NST - 1 || p.Kpad % KW != 0 || lds > 160 * 1024 ||
      (size_t)p.M * p.ldy * 4 >= (1ull << 31))
    return false;
  const bool cbig = (p.C % KW) == 0;
  static bool once = false;
  if (!once) {
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, true, OCC, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, OCC, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, true, OCC, true>);
    p3_set_lds_once(conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, OCC, true>);
    once = true;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int ntiles = ((p.M + BM - 1) / BM) * ((p.Nout + BN - 1) / BN);
  const long long T = (long long)ntiles * nk;
  const int per_cu = (int)((160 * 1024) / lds) < OCC ? (int)((160 * 1024) / lds) : OCC;
  const int slots = cus * (per_cu > 0 ? per_cu : 1);
  const int grid = (int)(T < slots ? T : slots);
  if ((T + 1) * grid >= (1ll << 32)) return false;  // the kernel's share arithmetic is 32-bit
  // shares of any tile: the shares meeting nk consecutive iterations, each share >= T / grid long
  const int smax = (int)((nk - 1) / (T / grid) + 2);
  if ((long long)ntiles * smax * BM * BN > p.ws_floats || ntiles > p.cnt_n) return false;
  p.splits = smax;
  static const bool probe = getenv("HCB_SK_PROBE") != nullptr && getenv("HCB_SK_PROBE")[0] == '1';
  if (probe) p.cnt = nullptr;  // tools/diag/sk_probe.sh: the main loop alone, hand-offs skipped (wrong output)
  const dim3 b(WM * WN * 64);
  if (cbig && stats)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, true, OCC, true>), dim3(grid), b, lds, st,
                       p);
  else if (cbig)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, true, false, OCC, true>), dim3(grid), b, lds,
                       st, p);
  else if (stats)
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, true, OCC, true>), dim3(grid), b, lds,
                       st, p);
  else
    hipLaunchKernelGGL((conv_p3_persist_kernel<WM, WN, TM, TN, KW, NST, false, false, OCC, true>), dim3(grid), b, lds,
                       st, p);
  return true;
}

}  // namespace hcb

namespace hcb {

// ============================================================== persistent weight gradient
// The weight-gradient plane GEMM (conv_p3_wgrad.h) as a persistent kernel: a workgroup walks the
// (tile, split) work items first, first + grid, ... with its LDS-DMA ring running across item
// boundaries, and adds each finished item into dW straight from the accumulator registers (one
// buffer atomic per element; masked elements add to an out-of-range offset, so every epilogue is
// exactly EOPS vector-memory instructions and the ring's vmcnt waits stay compile-time counts, as
// in conv_p3_persist_kernel). One atomic per element and item: with one split (the deterministic
// mode) every element receives a single add. NST = 2 only: the last split of a tile may own a
// single 32-row k-step, and the wait arithmetic allows one epilogue per window of NST-1 steps.
template <int WM, int WN, int TM, int TN, bool CBIG, int OCC>
__global__ __launch_bounds__(WM* WN * 64, OCC* WM* WN / 4) void conv_wgrad_p3_persist_kernel(WgradParams p, int nsplit) {
  constexpr int NST = 2, BK = 32;
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;
  constexpr int ARPI = 64 / ACPR, BRPI = 64 / BCPR;
  constexpr int AI = BK / ARPI / NW, BI = BK / BRPI / NW;
  constexpr int LOADS = NPL * (AI + BI);
  constexpr int AIMG = BK * BM * 2, BIMG = BK * BN * 2;
  constexpr int STAGE = NPL * (AIMG + BIMG);
  constexpr int EOPS = MI * NI * 4;
  static_assert(AI * ARPI * NW == BK && BI * BRPI * NW == BK && AI >= 1 && BI >= 1, "tile / wave mapping");
  static_assert(LOADS * (NST - 1) + EOPS <= 63 && NST * STAGE <= 160 * 1024, "vmcnt range / ring");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = (p.Nout + BM - 1) / BM;
  const int tiles_n = (p.K + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int items = ntiles * nsplit;
  const int grid = gridDim.x;
  const int first = xcd_remap(blockIdx.x, grid);
  if (first >= items) return;  // uniform
  const int mine = (items - 1 - first) / grid + 1;
  const int rows_per = p.ksteps_per_split * 64;

  const char* db = reinterpret_cast<const char*>(p.dy);
  const char* xb = reinterpret_cast<const char*>(p.x);
  const __amdgpu_buffer_rsrc_t dyr0 = make_rsrc(db, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t dyr1 = make_rsrc(db + p.dy_plane, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t dyr2 = make_rsrc(db + 2 * (size_t)p.dy_plane, p.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr0 = make_rsrc(xb, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr1 = make_rsrc(xb + p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr2 = make_rsrc(xb + 2 * (size_t)p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t dwr = make_rsrc(p.dw, (uint32_t)((size_t)p.Nout * p.K * 4));

  // per-thread LDS image positions (fixed) and the column chunk each lane fetches
  int a_row[AI], a_chunk[AI], b_row[BI], b_chunk[BI];
#pragma unroll
  for (int v = 0; v < AI; ++v) {
    const int row = (wid * AI + v) * ARPI + lane / ACPR, pos = lane % ACPR;
    a_row[v] = row;
    a_chunk[v] = (((pos >> 1) ^ p3w_swz<BM / 16>(row)) << 1) | (pos & 1);
  }
#pragma unroll
  for (int v = 0; v < BI; ++v) {
    const int row = (wid * BI + v) * BRPI + lane / BCPR, pos = lane % BCPR;
    b_row[v] = row;
    b_chunk[v] = (((pos >> 1) ^ p3w_swz<BN / 16>(row)) << 1) | (pos & 1);
  }
  auto item_rows = [&](int i, int& mbeg, int& mend) {
    const int t = first + i * grid;
    const int split = t / ntiles;
    mbeg = split * rows_per;
    mend = min(mbeg + rows_per, p.M);
  };

  // ---- issue cursor (item ci, k-step ck)
  int ci = 0, ck = 0, c_nk = 0, c_mbeg = 0, c_mend = 0;
  int a_col[AI], b_c[BI], b_dh[BI], b_dw[BI];
  bool b_ok[BI];
  auto cursor_item = [&](int i) {
    const int t = first + i * grid;
    const int tile = t % ntiles;
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int i0 = tm * BM, j0 = tn * BN;
    item_rows(i, c_mbeg, c_mend);
    c_nk = (c_mend - c_mbeg + BK - 1) / BK;
#pragma unroll
    for (int v = 0; v < AI; ++v) a_col[v] = i0 + a_chunk[v] * 8;
#pragma unroll
    for (int v = 0; v < BI; ++v) {
      const int col = j0 + b_chunk[v] * 8;
      int tap, c;
      if constexpr (CBIG) {
        tap = j0 / p.C;
        c = j0 - tap * p.C + b_chunk[v] * 8;
      } else {
        tap = (int)fdiv((uint32_t)col, p.fd_c);
        c = col - tap * p.C;
      }
      const int r = (int)fdiv((uint32_t)tap, p.fd_s), s = tap - r * p.S;
      b_c[v] = c;
      b_dh[v] = r * p.dil_h - p.pad_h;
      b_dw[v] = s * p.dil_w - p.pad_w;
      b_ok[v] = col < p.K;
    }
  };
  cursor_item(0);
  auto issue = [&](int stage) {
    const bool live = ci < mine;
    const int mb = c_mbeg + ck * BK;
    char* sA = smem + stage * STAGE;
    char* sB = sA + NPL * AIMG;
#pragma unroll
    for (int v = 0; v < AI; ++v) {
      const int m = mb + a_row[v];
      const bool ok = live & (a_col[v] < p.Nout) & (m < c_mend);
      const uint32_t off = ((uint32_t)(m * p.ldy + a_col[v]) * 2u) | ((uint32_t)!ok << 31);
      char* d = sA + (wid * AI + v) * ARPI * BM * 2;
      glds16(dyr0, d, off);
      glds16(dyr1, d + AIMG, off);
      glds16(dyr2, d + 2 * AIMG, off);
    }
#pragma unroll
    for (int v = 0; v < BI; ++v) {
      const int m = mb + b_row[v];
      const int n = (int)fdiv((uint32_t)m, p.fd_pq);
      const int rem = m - n * p.P * p.Q;
      const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
      const int qq = rem - pp * p.Q;
      const int h = pp * p.stride_h + b_dh[v], w = qq * p.stride_w + b_dw[v];
      const bool ok = live & b_ok[v] & (m < c_mend) & ((unsigned)h < (unsigned)p.H) & ((unsigned)w < (unsigned)p.W);
      const uint32_t raw = (uint32_t)(((n * p.H + h) * p.W + w) * p.ldx + b_c[v]) * 2u;
      const uint32_t off = raw | ((uint32_t)!ok << 31);
      char* d = sB + (wid * BI + v) * BRPI * BN * 2;
      glds16(xr0, d, off);
      glds16(xr1, d + BIMG, off);
      glds16(xr2, d + 2 * BIMG, off);
    }
  };
  auto advance = [&]() {
    if (++ck == c_nk) {
      ck = 0;
      if (++ci < mine) cursor_item(ci);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, g = lane >> 4, q4 = li >> 2, p4 = li & 3;
  auto epilogue = [&](int i) {
    const int t = first + i * grid;
    const int tile = t % ntiles;
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int rbase = tm * BM + wm * TM + g * 4, cbase = tn * BN + wn * TN + li;
#pragma unroll
    for (int ii = 0; ii < MI; ++ii)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + ii * 16 + e;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int col = cbase + j * 16;
          const bool ok = (row < p.Nout) & (col < p.K);
          buf_atomic_add_f32(dwr, ok ? (uint32_t)(row * p.K + col) * 4u : HCB_OOB, acc[ii][j][e]);
        }
      }
#pragma unroll
    for (int ii = 0; ii < MI; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // transposed fragment reads, as conv_wgrad_p3_kernel
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
  using Fr = P3Frags<TM, TN, 1>;
  auto read = [&](int gstep, Fr& f) {
    const char* Ab = smem + (gstep % NST) * STAGE;
    const char* Bb = Ab + NPL * AIMG;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int t = 0; t < NPL; ++t) f.a[0][t][i] = frag(Ab + t * AIMG, BM, 8 * g, wm * TM + i * 16);
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int t = 0; t < NPL; ++t) f.b[0][t][j] = frag(Bb + t * BIMG, BN, 8 * g, wn * TN + j * 16);
  };

#pragma unroll
  for (int s = 0; s < NST; ++s) {
    issue(s);
    advance();
  }
  int nsteps = 0;
  for (int i = 0; i < mine; ++i) {
    int mb, me;
    item_rows(i, mb, me);
    nsteps += (me - mb + BK - 1) / BK;
  }
  int i = 0, k = 0, nk_cur;
  {
    int mb, me;
    item_rows(0, mb, me);
    nk_cur = (me - mb + BK - 1) / BK;
  }
  auto post = [&]() {
    if (++k == nk_cur) {
      epilogue(i);
      k = 0;
      if (++i < mine) {
        int mb, me;
        item_rows(i, mb, me);
        nk_cur = (me - mb + BK - 1) / BK;
      }
    }
  };
  constexpr int FREGS = (MI + NI) * NPL * 4, AREGS = MI * NI * 4;
  constexpr int RBUDGET = p3_regs_per_wave<OCC, NW>() - 88 < 400 ? p3_regs_per_wave<OCC, NW>() - 88 : 400;
  constexpr bool PIPE = 2 * FREGS + AREGS <= RBUDGET;
  constexpr int NMF = MI * NI * 6, NRD = 2 * (MI + NI) * NPL;
  if constexpr (PIPE) {
    Fr fr[2];
    wait_vmcnt<(NST - 1) * LOADS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, fr[0]);
    auto body = [&](int gs, Fr& cur, Fr& nxt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (i > 0 && k == 0)  // the previous item's epilogue was issued after slot gs+1's DMA
        wait_vmcnt<EOPS>();
      else
        wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(gs % NST);
      read(gs + 1, nxt);
      p3_mma<TM, TN, 1>(cur, acc);
      ilv_schedule<NMF, LOADS, NRD>();
      advance();
      post();
    };
    for (int gs = 0; gs < nsteps; gs += 2) {
      body(gs, fr[0], fr[1]);
      if (gs + 1 < nsteps) body(gs + 1, fr[1], fr[0]);
    }
  } else {
    Fr fr;
    for (int gs = 0; gs < nsteps; ++gs) {
      // slot gs landed: one later slot issue, plus an epilogue issued after slot gs's DMA (the first
      // two steps of an item; two epilogues in the window only make the count conservative)
      if (i > 0 && k <= 1)
        wait_vmcnt<LOADS + EOPS>();
      else
        wait_vmcnt<LOADS>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read(gs, fr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(gs % NST);
      p3_mma<TM, TN, 1>(fr, acc);
      ilv_schedule<NMF, LOADS, 0>();
      advance();
      post();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy pieces have landed before the LDS is freed
}

template <int WM, int WN, int TM, int TN, int OCC>
static void wlaunch_p3p(const WgradParams& p, int splits, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  const int tiles = ((p.Nout + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  const size_t lds = (size_t)2 * NPL * 32 * (BM + BN) * 2;
  static bool once = false;
  if (!once) {
    p3_set_lds_once(conv_wgrad_p3_persist_kernel<WM, WN, TM, TN, true, OCC>);
    p3_set_lds_once(conv_wgrad_p3_persist_kernel<WM, WN, TM, TN, false, OCC>);
    once = true;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int items = tiles * splits;
  const int per_cu = (int)((160 * 1024) / lds) < OCC ? (int)((160 * 1024) / lds) : OCC;
  const int slots = cus * (per_cu > 0 ? per_cu : 1);
  const int grid = items < slots ? items : slots;
  const dim3 b(WM * WN * 64);
  if ((p.C % BN) == 0)
    hipLaunchKernelGGL((conv_wgrad_p3_persist_kernel<WM, WN, TM, TN, true, OCC>), dim3(grid), b, lds, st, p, splits);
  else
    hipLaunchKernelGGL((conv_wgrad_p3_persist_kernel<WM, WN, TM, TN, false, OCC>), dim3(grid), b, lds, st, p, splits);
}

}  // namespace hcb
