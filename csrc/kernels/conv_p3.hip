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
#include "conv_p3_persist.h"
#include "conv_p3_wgrad.h"

namespace hcb {

// cfg 0-17: conv_igemm_p3_kernel (conv_p3_fwd.h); 18-22: the persistent short-K kernel
// (conv_p3_persist.h), twins of 15, 14, 16, 17 and 7; 23-27: its stream-K form (tiles of 18-22);
// 28: stream-K with cfg 8's geometry (4 x 2 waves of 32 x 64); 29 / 30 (stream-K 256 x 128 / 128 x 256
// of 64 x 64 wave tiles) are retired -- a 272-byte stack frame, 5x slower (profiles/r6_quantization_streamk.txt)
// -- and launch cfg 10 / 11
// 31-36: the persistent kernel with the workgroup's weight slice resident in LDS (BRES): 64x256 (4
// waves of 64x64), 128x256 (8 waves of 64x64), 64x64 (4 waves of 32x32), 128x64 (4 waves of 64x32),
// 128x64 (8 waves of 32x32), 128x128 (8 waves of 32x64)
constexpr int N_P3_CFG = 37;
int p3_tile_m(int cfg) {
  static const int t[N_P3_CFG] = {128, 64, 128, 64, 64, 128, 64, 128, 128, 128, 256, 128, 64, 128, 128, 64,
                                  64, 64, 64, 128, 64, 64, 128, 64, 128, 64, 64, 128, 128, 256, 128,
                                  64, 128, 64, 128, 128, 128};
  return (cfg >= 0 && cfg < N_P3_CFG) ? t[cfg] : 128;
}
int p3_slot_k(int cfg) { return (cfg >= 0 && cfg <= 6) ? 64 : 32; }
int p3_tile_n(int cfg) {
  static const int t[N_P3_CFG] = {64, 128, 64, 128, 64, 64, 128, 128, 128, 128, 128, 256, 128, 64, 64, 128,
                                  64, 64, 128, 64, 64, 64, 128, 128, 64, 64, 64, 128, 128, 128, 256,
                                  256, 256, 64, 64, 64, 128};
  return (cfg >= 0 && cfg < N_P3_CFG) ? t[cfg] : 64;
}

// the persistent cfg, or (a problem with an epilogue it does not serve) its twin; the stream-K cfg,
// else its whole-tile persistent form
static int launch_p3_persist(const ConvParams& p, int cfg, hipStream_t st) {
  switch (cfg) {
    case 23: return launch_p3sk<2, 2, 32, 64, 32, 2, 2>(p, st) ? -1 : launch_p3_persist(p, 18, st);
    case 24: return launch_p3sk<2, 2, 64, 32, 32, 2, 2>(p, st) ? -1 : launch_p3_persist(p, 19, st);
    case 25: return launch_p3sk<2, 2, 32, 32, 32, 3, 2>(p, st) ? -1 : launch_p3_persist(p, 20, st);
    case 26: return launch_p3sk<2, 2, 32, 32, 32, 2, 3>(p, st) ? -1 : launch_p3_persist(p, 21, st);
    case 27: return launch_p3sk<2, 4, 64, 32, 32, 3, 1>(p, st) ? -1 : launch_p3_persist(p, 22, st);
    case 28: return launch_p3sk<4, 2, 32, 64, 32, 3, 1>(p, st) ? -1 : 8;
    case 29: return 10;
    case 30: return 11;
    case 31: return launch_p3bres<1, 4, 64, 64, 32, 3>(p, st) ? -1 : launch_p3_persist(p, 18, st);
    case 32: return launch_p3bres<2, 4, 64, 64, 32, 2>(p, st) ? -1 : launch_p3_persist(p, 18, st);
    case 33: return launch_p3bres<2, 2, 32, 32, 32, 3>(p, st) ? -1 : launch_p3_persist(p, 20, st);
    case 34: return launch_p3bres<2, 2, 64, 32, 32, 2>(p, st) ? -1 : launch_p3_persist(p, 19, st);
    case 35: return launch_p3bres<4, 2, 32, 32, 32, 2>(p, st) ? -1 : launch_p3_persist(p, 19, st);
    case 36: return launch_p3bres<4, 2, 32, 64, 32, 2>(p, st) ? -1 : launch_p3_persist(p, 22, st);
    case 18: return launch_p3p<2, 2, 32, 64, 32, 2, 2>(p, st) ? -1 : 15;
    case 19: return launch_p3p<2, 2, 64, 32, 32, 2, 2>(p, st) ? -1 : 14;
    case 20: return launch_p3p<2, 2, 32, 32, 32, 3, 2>(p, st) ? -1 : 16;
    case 21: return launch_p3p<2, 2, 32, 32, 32, 2, 3>(p, st) ? -1 : 17;
    case 22: return launch_p3p<2, 4, 64, 32, 32, 3, 1>(p, st) ? -1 : 7;
    default: return cfg;
  }
}

void set_p3p_bnb(int v) { p3p_bnb_level() = v; }

void launch_conv_p3(const ConvParams& p, int cfg, hipStream_t st) {
  if (cfg >= 18 && (cfg = launch_p3_persist(p, cfg, st)) < 0) return;
  if (p.bnb_acc != nullptr)
    launch_p3_cfg<true>(p, cfg, st);
  else
    launch_p3_cfg<false>(p, cfg, st);
}
// p3 wgrad cfg (block tile, waves x wave tile, slots x pixel rows):
//   0 128x64 (2x2 of 64x32, 2x64), 1 64x128 (2x2 of 32x64, 2x64), 2 64x64 (2x2 of 32x32, 3x64),
//   3 128x64 (4x2 of 32x32, 2x64), 4 64x128 (2x4 of 32x32, 2x64), 5 64x64 (2x2 of 32x32, 2x64),
//   6 128x128 (2x4 of 64x32, 3x32), 7 128x128 (4x2 of 32x64, 3x32), 8 256x128 (4x2 of 64x64, 2x32),
//   9 128x256 (2x4 of 64x64, 2x32), 10 128x128 (2x2 of 64x64, 3x32), 11 128x64 (2x2 of 64x32, 3x32),
//   two per CU: 12 128x64 (2x2 of 64x32, 2x32), 13 64x128 (2x2 of 32x64, 2x32), 14 64x64 (2x2 of 32x32, 3x32),
//   three per CU: 15 64x64 (2x2 of 32x32, 2x32)
//   persistent (conv_p3_persist.h, twins of 12, 13, 15): 16 128x64, 17 64x128, 18 64x64
constexpr int N_WP3_CFG = 19;
int wgrad_p3_tile_m(int cfg) {
  static const int t[N_WP3_CFG] = {128, 64, 64, 128, 64, 64, 128, 128, 256, 128, 128, 128, 128, 64, 64, 64, 128, 64, 64};
  return (cfg >= 0 && cfg < N_WP3_CFG) ? t[cfg] : 64;
}
int wgrad_p3_tile_n(int cfg) {
  static const int t[N_WP3_CFG] = {64, 128, 64, 64, 128, 64, 128, 128, 128, 256, 128, 64, 64, 128, 64, 64, 64, 128, 64};
  return (cfg >= 0 && cfg < N_WP3_CFG) ? t[cfg] : 64;
}

void launch_wgrad_p3(const WgradParams& p, int cfg, int splits, hipStream_t st) {
  switch (cfg) {
    case 16: wlaunch_p3p<2, 2, 64, 32, 2>(p, splits, st); break;
    case 17: wlaunch_p3p<2, 2, 32, 64, 2>(p, splits, st); break;
    case 18: wlaunch_p3p<2, 2, 32, 32, 3>(p, splits, st); break;
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
