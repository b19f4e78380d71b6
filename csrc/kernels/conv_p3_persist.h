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
#include "conv_p3_fwd.h"

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

// STATS: BN statistics into p.stats_R replicas. WM <= 2: a replica slot of a tile receives one add
// per wave row, and two fp32 adds commute exactly, so the deterministic mode's one-replica-per-tile
// statistics stay bitwise reproducible.
template <int WM, int WN, int TM, int TN, int KW, int NST, bool CBIG, bool STATS, int OCC>
__global__ __launch_bounds__(WM* WN * 64, OCC* WM* WN / 4) void conv_p3_persist_kernel(ConvParams p) {
  constexpr int BM = WM * TM, BN = WN * TN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int NT = WM * WN * 64, CPR = KW / 8, RB = KW * 2;
  constexpr int RP = NT / CPR;
  constexpr int AV = BM / RP, BV = BN / RP;
  constexpr int LOADS = NPL * (AV + BV);
  constexpr int AIMG = BM * RB, BIMG = BN * RB;
  constexpr int STAGE = (int)p3_stage_bytes<BM, BN, KW>();
  constexpr int EOPS = MI * NI * 4 + (STATS ? 2 * NI : 0);  // epilogue vector-memory instructions
  static_assert(WM <= 2, "at most two adds per statistics slot and tile (deterministic mode)");
  static_assert(AV * RP == BM && BV * RP == BN, "tile rows must be a multiple of the load pass");
  static_assert(LOADS * (NST - 1) + EOPS <= 63 && NST >= 2 && NST <= 4, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* ktab = reinterpret_cast<float*>(smem + p3p_ring_bytes<BM, BN, KW, NST>());

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = wave_id_uniform();
  const int wm = wid / WN, wn = wid % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int tiles_n = (p.Nout + BN - 1) / BN;
  const int ntiles = ((p.M + BM - 1) / BM) * tiles_n;
  const int grid = gridDim.x;
  const int first = xcd_remap(blockIdx.x, grid);  // concurrent neighbours (same M rows) share an XCD
  if (first >= ntiles) return;                     // uniform (the host sizes grid <= ntiles)
  const int mine = (ntiles - 1 - first) / grid + 1;
  const int nk = p.Kpad / KW;
  const int chunk = (tid % CPR) ^ p3_swz<KW>(tid / CPR);

  const char* xb = reinterpret_cast<const char*>(p.x);
  const __amdgpu_buffer_rsrc_t xr0 = make_rsrc(xb, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr1 = make_rsrc(xb + p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t xr2 = make_rsrc(xb + 2 * (size_t)p.x_plane, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr0 = make_rsrc(p.w, p.w_bytes);
  const __amdgpu_buffer_rsrc_t wr1 = make_rsrc(p.w_lo, p.w_bytes);
  const __amdgpu_buffer_rsrc_t wr2 = make_rsrc(p.w_lo2, p.w_bytes);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, (uint32_t)((size_t)p.M * p.ldy * 4));
  const __amdgpu_buffer_rsrc_t sr = make_rsrc(p.stats, STATS ? (uint32_t)((size_t)p.stats_R * 2 * p.Nout * 4) : 0u);

  if constexpr (STATS) {  // published by the first barrier; older than every DMA (vmcnt order)
    for (int c = tid; c < p.Nout; c += NT) ktab[c] = p.stats_shift != nullptr ? p.stats_shift[c] : 0.f;
  }

  // ---- issue cursor: the (local tile, k-step) whose slot is issued next, NST steps ahead of the
  // MFMAs; its loader state follows it across tile boundaries
  ALoader<AV, CBIG, false, RP, 2, KW> al;
  uint32_t b_off[BV];
  int ci = 0, ck = 0;
  auto cursor_tile = [&](int i) {
    const int t = first + i * grid;
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    al.init(p, tm * BM, tid, chunk);
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int j = tn * BN + tid / CPR + RP * v;
      b_off[v] = (j < p.Nout) ? (uint32_t)(j * p.Kpad + chunk * 8) * 2u : HCB_OOB;
    }
  };
  cursor_tile(0);
  constexpr int WROWS = 64 / CPR;
  // branch-free: past the last tile every piece is out of range (lands zeros in a slot nobody reads)
  auto issue = [&](int stage) {
    const bool live = ci < mine;
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
    char* sb = smem + stage * STAGE + NPL * AIMG + wid * WROWS * RB;
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const uint32_t o = (b_off[v] == HCB_OOB || !live) ? HCB_OOB : b_off[v] + (uint32_t)ck * (uint32_t)RB;
      glds16(wr0, sb + RP * v * RB, o);
      glds16(wr1, sb + BIMG + RP * v * RB, o);
      glds16(wr2, sb + 2 * BIMG + RP * v * RB, o);
    }
  };
  auto advance = [&]() {
    if (++ck == nk) {
      ck = 0;
      if (++ci < mine) cursor_tile(ci);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- register epilogue of local tile i: exactly EOPS vector-memory instructions per thread
  auto epilogue = [&](int i) {
    const int t = first + i * grid;
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    const int rbase = tm * BM + wm * TM;           // the wave's first row
    const int cbase = tn * BN + wn * TN + frow;    // the lane's column in fragment j = 0
    if constexpr (STATS) {
      const int wrows = p.M - rbase;
      const uint32_t rep = (uint32_t)(tm % p.stats_R) * 2u * (uint32_t)p.Nout;
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
#pragma unroll
    for (int ii = 0; ii < MI; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto read = [&](int g, P3Frags<TM, TN, KW / 32>& f) {
    const char* sb = smem + (g % NST) * STAGE;
    p3_read<WM, WN, TM, TN, KW>(reinterpret_cast<const u32x4*>(sb), reinterpret_cast<const u32x4*>(sb + NPL * AIMG), f,
                                wm, wn, lane);
  };

#pragma unroll
  for (int s = 0; s < NST; ++s) {
    issue(s);
    advance();
  }
  const int nsteps = mine * nk;
  constexpr int FREGS = (MI + NI) * NPL * 4 * (KW / 32), AREGS = MI * NI * 4;
  constexpr int RBUDGET = p3_regs_per_wave<OCC, WM * WN>() - 64 < 400 ? p3_regs_per_wave<OCC, WM * WN>() - 64 : 400;
  constexpr bool PIPE = 2 * FREGS + AREGS <= RBUDGET;
  constexpr int NMF = (KW / 32) * MI * NI * 6, NRD = (KW / 32) * (MI + NI) * NPL;
  int i = 0, k = 0;  // the compute side's local tile and k-step
  // after the MFMAs of step g: the tile's epilogue once its last k-step is in
  auto post = [&]() {
    if (++k == nk) {
      epilogue(i);
      k = 0;
      ++i;
    }
  };
  if constexpr (PIPE) {
    P3Frags<TM, TN, KW / 32> fr[2];
    wait_vmcnt<(NST - 1) * LOADS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, fr[0]);
    auto body = [&](int g, P3Frags<TM, TN, KW / 32>& cur, P3Frags<TM, TN, KW / 32>& nxt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot g are done
      // slot g+1 has landed for this thread
      if (i > 0 && k <= NST - 2)
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
      post();
    };
    for (int g = 0; g < nsteps; g += 2) {
      body(g, fr[0], fr[1]);
      if (g + 1 < nsteps) body(g + 1, fr[1], fr[0]);
    }
  } else {
    P3Frags<TM, TN, KW / 32> fr;
    for (int g = 0; g < nsteps; ++g) {
      // slot g has landed: NST-1 later slot issues, plus the previous epilogue when it came after
      if (i > 0 && k <= NST - 1)
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
      post();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy pieces have landed before the LDS is freed
}

// cfg 18-22 (persistent twins of cfg 15, 14, 16, 17, 7): false when the problem needs an epilogue
// feature this kernel does not have (the caller then launches the twin)
template <int WM, int WN, int TM, int TN, int KW, int NST, int OCC>
static bool launch_p3p(const ConvParams& p, hipStream_t st) {
  constexpr int BM = WM * TM, BN = WN * TN;
  const bool stats = p.stats != nullptr;
  const int nk = p.Kpad / KW;
  const size_t ring = p3p_ring_bytes<BM, BN, KW, NST>();
  const size_t lds = ring + (stats ? (size_t)p.Nout * 4 : 0);
  if (p.bnb_acc != nullptr || p.remap || p.idil_h > 1 || p.idil_w > 1 || p.splits != 1 || p.beta ||
      p.bias != nullptr || !p.out_f32 ||
      (stats && p.stats_R <= 0) || nk < NST - 1 || p.Kpad % KW != 0 || lds > 160 * 1024 ||
      (size_t)p.M * p.ldy * 4 >= (1ull << 31))
    return false;
  const bool cbig = (p.C % KW) == 0;
  static bool once = false;
  if (!once) {
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
  if (cbig && stats)
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

}  // namespace hcb
