// ResNet stem (7x7/2 conv on 3-channel 224x224 images; the reference's first MKL-DNN conv,
// SURVEY.md §2.6 row 1) as a space-to-depth 4x4/1 implicit GEMM.
//
// The direct form gathers 7*7 taps of an 8-channel (3 real + 5 zero) input: K = 392 -> 448,
// 2.67x the 147 useful MACs per output. Folding 2x2 input pixels into channels turns the
// stride-2 7x7 conv into a stride-1 4x4 conv on a [N][H/2+3][W/2+3][16] tensor:
//
//   out(p,q) = sum_{i,j<4} sum_{a,b<2} X'(p+i, q+j, (2a+b)*4 + c) W'(i, j, (2a+b)*4 + c)
//   X'(P, Q, (2a+b)*4 + c) = x(2P + a - 4, 2Q + b - 4, c)            (c < 4; zero outside)
//   W'(i, j, (2a+b)*4 + c) = w(2i + a - 1, 2j + b - 1, c)             (zero outside 7x7, c >= 3)
//
// so K = 16 taps x 16 channels = 256 (every 16-byte vector still holds 8 channels of one tap),
// 1.75x fewer MACs than the padded direct form. Three small kernels surround the ordinary
// implicit-GEMM kernels: the input fold (per step), the weight fold (per step, from the fp32
// master) and the scatter of the folded weight gradient back into the master layout.
#include "common.h"
#include "kernels.h"

namespace hcb {

// one thread per folded pixel: 4 source pixels x 4 channels (8 bytes each) -> 32 bytes
__global__ __launch_bounds__(256) void stem_s2d_kernel(const uint16_t* __restrict__ x, int N, int H, int W, int ldx,
                                                       uint16_t* __restrict__ out, int Hs, int Ws, int pad) {
  const int64_t total = (int64_t)N * Hs * Ws;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int Q = (int)(t % Ws);
    const int64_t r = t / Ws;
    const int P = (int)(r % Hs);
    const int n = (int)(r / Hs);
    u32x2 v[4];
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) {
      const int h = 2 * P + (ab >> 1) - pad, w = 2 * Q + (ab & 1) - pad;
      if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
        v[ab] = *reinterpret_cast<const u32x2*>(x + (((int64_t)n * H + h) * W + w) * ldx);
      else
        v[ab] = u32x2{0u, 0u};
    }
    u32x4* o = reinterpret_cast<u32x4*>(out + t * 16);
    o[0] = u32x4{v[0][0], v[0][1], v[1][0], v[1][1]};
    o[1] = u32x4{v[2][0], v[2][1], v[3][0], v[3][1]};
  }
}

// fp32 path: the fold straight from the fp32 image into the three bf16 planes of the folded
// tensor (plane stride `plane` elements): the split of each value (split3_8) happens here, so the
// image is read once and no full-size planes copy of it is written and re-read
__global__ __launch_bounds__(256) void stem_s2d_f32_kernel(const float* __restrict__ x, int N, int H, int W, int ldx,
                                                           uint16_t* __restrict__ out, int64_t plane, int Hs, int Ws,
                                                           int pad) {
  const int64_t total = (int64_t)N * Hs * Ws;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int Q = (int)(t % Ws);
    const int64_t r = t / Ws;
    const int P = (int)(r % Hs);
    const int n = (int)(r / Hs);
    u32x4 v[4];
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) {
      const int h = 2 * P + (ab >> 1) - pad, w = 2 * Q + (ab & 1) - pad;
      if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
        v[ab] = *reinterpret_cast<const u32x4*>(x + (((int64_t)n * H + h) * W + w) * ldx);
      else
        v[ab] = u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {  // source pixels (0, 1), then (2, 3): 8 values each
      u32x4 hi, mid, lo;
      split3_8(v[2 * hf], v[2 * hf + 1], hi, mid, lo);
      uint16_t* o = out + t * 16 + hf * 8;
      *reinterpret_cast<u32x4*>(o) = hi;
      *reinterpret_cast<u32x4*>(o + plane) = mid;
      *reinterpret_cast<u32x4*>(o + 2 * plane) = lo;
    }
  }
}

// folded bf16 GEMM operand W'[cout][256] from the fp32 master w[cout][7][7][cs] (cs = stored
// channels, the first 3 real)
// P3 (fp32 path): the folded weight as bf16 hi / mid / lo planes (plane stride cout * 256)
template <bool P3>
__global__ __launch_bounds__(256) void stem_wfold_kernel(const float* __restrict__ w, int cout, int cs,
                                                         uint16_t* __restrict__ wp) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cout * 256) return;
  const int k = t >> 8, e = t & 255;
  const int tap = e >> 4, cc = e & 15;
  const int i = tap >> 2, j = tap & 3, a = cc >> 3, b = (cc >> 2) & 1, c = cc & 3;
  const int r = 2 * i + a - 1, s = 2 * j + b - 1;
  float v = 0.f;
  if ((unsigned)r < 7u && (unsigned)s < 7u && c < 3) v = w[((k * 7 + r) * 7 + s) * cs + c];
  if constexpr (P3) {
    const int n = cout * 256;
    const float h = bf2f(f2bf(v)), rr = v - h, m = bf2f(f2bf(rr));
    wp[t] = f2bf(v);
    wp[n + t] = f2bf(rr);
    wp[2 * n + t] = f2bf(rr - m);
  } else {
    wp[t] = f2act(v);
  }
}

// dw[cout][7][7][cs] += dW'[cout][256] mapped back (each real weight has exactly one folded slot)
__global__ __launch_bounds__(256) void stem_wgrad_unfold_kernel(const float* __restrict__ dwp, int cout, int cs,
                                                                float* __restrict__ dw) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cout * 49 * 3) return;
  const int c = t % 3, rs = (t / 3) % 49, k = t / 147;
  const int r = rs / 7, s = rs % 7;
  const int i = (r + 1) >> 1, a = (r + 1) & 1, j = (s + 1) >> 1, b = (s + 1) & 1;
  dw[((k * 7 + r) * 7 + s) * cs + c] += dwp[k * 256 + (i * 4 + j) * 16 + (2 * a + b) * 4 + c];
}

void launch_stem_s2d(const uint16_t* x, int N, int H, int W, int ldx, uint16_t* out, int Hs, int Ws, int pad,
                     hipStream_t st) {
  const int64_t total = (int64_t)N * Hs * Ws;
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(stem_s2d_kernel, dim3((int)g), dim3(256), 0, st, x, N, H, W, ldx, out, Hs, Ws, pad);
}
void launch_stem_s2d_f32(const float* x, int N, int H, int W, int ldx, uint16_t* out, int64_t plane, int Hs, int Ws,
                         int pad, hipStream_t st) {
  const int64_t total = (int64_t)N * Hs * Ws;
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(stem_s2d_f32_kernel, dim3((int)g), dim3(256), 0, st, x, N, H, W, ldx, out, plane, Hs, Ws, pad);
}
void launch_stem_wfold(const float* w, int cout, int cs, uint16_t* wp, hipStream_t st, bool p3) {
  if (p3)
    hipLaunchKernelGGL(stem_wfold_kernel<true>, dim3((cout * 256 + 255) / 256), dim3(256), 0, st, w, cout, cs, wp);
  else
    hipLaunchKernelGGL(stem_wfold_kernel<false>, dim3((cout * 256 + 255) / 256), dim3(256), 0, st, w, cout, cs, wp);
}
void launch_stem_wgrad_unfold(const float* dwp, int cout, int cs, float* dw, hipStream_t st) {
  hipLaunchKernelGGL(stem_wgrad_unfold_kernel, dim3((cout * 147 + 255) / 256), dim3(256), 0, st, dwp, cout, cs, dw);
}

}  // namespace hcb
